"""Train the symmetric flip metric beta (mirror of dl_scl_polar/train/train_beta.py:64-177).

    python -m polar_code_amd.train.train_beta --M 4 --data 'data/ds*_part*.npz'

Same CLI, same algorithm and outputs: shards from make_dataset, a seeded NumPy split into
train/validation, logits = -(|L0| @ beta), cross-entropy to the labelled flip index plus
lambda * mean(off_diag^2), RMSprop; per-epoch CSV log ``{log_dir}/train_M{M}.csv`` and the
best-validation beta in ``{checkpoint_dir}/beta_M{M}.npy`` (float32 K x K, the format
run_fer_sweep --beta and pscl_set_beta take).  Runs on the GPU through PyTorch-ROCm unless
--cpu; on the CPU with one thread it reproduces the reference's checkpoint bit for bit.
"""
from __future__ import annotations

import argparse
import csv
from glob import glob
from pathlib import Path
from typing import Iterable, List, Tuple

import numpy as np
import torch
from torch import nn
from torch.utils.data import DataLoader, TensorDataset

from ..dlscl.beta import SymmetricBeta
from ..utils.seeding import seed_all


def load_shards(patterns: Iterable[str]) -> Tuple[np.ndarray, np.ndarray]:
    """Concatenate (abs_l0 float32, flip_idx int64) over the shards matched by each pattern."""
    xs, ys = [], []
    for pat in patterns:
        files = sorted(glob(pat)) or ([pat] if Path(pat).exists() else [])
        for f in files:
            z = np.load(f)  # plain arrays only (allow_pickle stays False)
            xs.append(z["abs_l0"])
            ys.append(z["flip_idx"])
    if not xs:
        raise FileNotFoundError("No dataset shards found for the provided --data patterns")
    return np.concatenate(xs).astype(np.float32), np.concatenate(ys).astype(np.int64)


def split(x: np.ndarray, y: np.ndarray, val_frac: float, seed: int):
    order = np.arange(x.shape[0])
    np.random.default_rng(seed).shuffle(order)
    cut = int(x.shape[0] * (1.0 - val_frac))
    part = lambda idx: TensorDataset(torch.from_numpy(x[idx]), torch.from_numpy(y[idx]))  # noqa: E731
    return part(order[:cut]), part(order[cut:])


def _epoch(model, loader, device, dim, lambda_l2, opt=None):
    """One pass; trains when an optimizer is given.  Returns (mean loss, accuracy, samples)."""
    ce = nn.CrossEntropyLoss()
    loss_sum, hits, n = 0.0, 0, 0
    for xb, yb in loader:
        xb, yb = xb.to(device), yb.to(device)
        if opt is not None:
            opt.zero_grad(set_to_none=True)
        logits = -model(xb)
        loss = ce(logits, yb)
        if opt is not None:
            if lambda_l2 > 0:
                loss = loss + lambda_l2 * (model.off_diag.pow(2).sum() / (dim * dim))
            loss.backward()
            model.clamp_diagonal()
            opt.step()
        loss_sum += loss.item() * xb.size(0)
        hits += (logits.argmax(dim=1) == yb).sum().item()
        n += xb.size(0)
    return loss_sum, hits, n


def train_beta(args: argparse.Namespace) -> Path:
    seed_all(args.seed)
    x, y = load_shards(args.data)
    dim = x.shape[1]
    train_ds, val_ds = split(x, y, args.val_frac, args.seed)
    train_dl = DataLoader(train_ds, batch_size=args.batch, shuffle=True)
    val_dl = DataLoader(val_ds, batch_size=args.batch, shuffle=False)
    device = torch.device("cuda" if (torch.cuda.is_available() and not args.cpu) else "cpu")
    model = SymmetricBeta(dim).to(device)
    opt = torch.optim.RMSprop(model.parameters(), lr=args.lr)

    log_dir, ckpt_dir = Path(args.log_dir), Path(args.checkpoint_dir)
    log_dir.mkdir(parents=True, exist_ok=True)
    ckpt_dir.mkdir(parents=True, exist_ok=True)
    ckpt = ckpt_dir / f"beta_M{args.M}.npy"
    best_val, best = float("inf"), None
    with (log_dir / f"train_M{args.M}.csv").open("w", newline="") as fh:
        log = csv.writer(fh)
        log.writerow(["epoch", "train_loss", "train_acc", "val_loss", "val_acc"])
        for epoch in range(1, args.epochs + 1):
            model.train()
            tl, th, tn = _epoch(model, train_dl, device, dim, args.lambda_l2, opt)
            model.eval()
            with torch.no_grad():
                vl, vh, vn = _epoch(model, val_dl, device, dim, args.lambda_l2)
            val_loss = vl / vn if vn else float("nan")
            val_acc = vh / vn if vn else float("nan")
            log.writerow([epoch, tl / max(tn, 1), th / max(tn, 1), val_loss, val_acc])
            fh.flush()
            if vn and val_loss < best_val:
                best_val, best = val_loss, model.beta_matrix().detach().cpu().numpy()
    if best is None:
        best = model.beta_matrix().detach().cpu().numpy()
    np.save(ckpt, best)
    print(f"Saved β checkpoint to {ckpt}")
    return ckpt


def build_argparser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Train symmetric β for DL-SCL")
    p.add_argument("--M", type=int, required=True, help="SCL list size")
    p.add_argument("--data", nargs="+", required=True, help="Glob(s) to dataset shards")
    p.add_argument("--epochs", type=int, default=8)
    p.add_argument("--lr", type=float, default=1e-4)
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--lambda_l2", type=float, default=0.25)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--val_frac", type=float, default=0.1)
    p.add_argument("--checkpoint_dir", type=str, default="checkpoints")
    p.add_argument("--log_dir", type=str, default="logs")
    p.add_argument("--cpu", action="store_true", help="Force CPU even if CUDA is available")
    return p


def main(argv: List[str] | None = None) -> None:
    train_beta(build_argparser().parse_args(argv))


if __name__ == "__main__":
    main()
