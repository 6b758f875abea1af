"""Learnable flip metric beta (mirror of dl_scl_polar/dlscl/beta.py:9-46).

beta = U + U^T + I, where U is the strict upper triangle of a dim x dim parameter (its
diagonal is kept at zero, the lower triangle is only touched by the training's L2 term).
q = |L0| @ beta ranks the flip candidates (flip.py:104-106).
"""
from __future__ import annotations

import torch
from torch import nn


class SymmetricBeta(nn.Module):
    def __init__(self, dim: int, init_range: float = 0.2) -> None:
        if dim <= 0:
            raise ValueError("dim must be positive")
        super().__init__()
        self.dim, self.init_range = dim, float(init_range)
        w = torch.empty(dim, dim)
        nn.init.uniform_(w, -self.init_range, self.init_range)  # U(-0.2, 0.2) off-diagonals
        w.fill_diagonal_(0.0)
        self.off_diag = nn.Parameter(w)

    def clamp_diagonal(self) -> None:
        """Keep the parameter's diagonal at zero (the unit diagonal is added in beta_matrix)."""
        with torch.no_grad():
            self.off_diag.fill_diagonal_(0.0)

    def beta_matrix(self) -> torch.Tensor:
        up = torch.triu(self.off_diag, diagonal=1)
        eye = torch.diag(torch.ones(self.dim, dtype=up.dtype, device=up.device))
        return (up + up.transpose(0, 1)) + eye

    def forward(self, abs_l0: torch.Tensor) -> torch.Tensor:
        if abs_l0.dim() not in (1, 2):
            raise ValueError("abs_l0 must be 1D or 2D tensor")
        return abs_l0 @ self.beta_matrix()


__all__ = ["SymmetricBeta"]
