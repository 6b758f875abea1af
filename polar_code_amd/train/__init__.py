"""Dataset labelling for beta training (mirror of dl_scl_polar/train)."""
