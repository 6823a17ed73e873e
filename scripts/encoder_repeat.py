"""Repeat the config-5 encoder forward in one process and bit-compare every run with the oracle
(determinism check for the encoder's launches; development aid, not a test)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _pkg  # noqa: E402
from oracle import oracle as O  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
qg = _pkg.package()
O.build()
seq, d, H, dff, blocks = 512, 1024, 16, 4096, 2
X = O.uniform((seq, d), 17)
ref = O.encoder_forward(X, d, H, dff, blocks, 19)
enc = qg.Encoder(d, H, dff, blocks, max_seq=seq, seed=19)
Xd = torch.from_numpy(X).cuda()
bad = 0
for r in range(reps):
    Y = enc.forward(Xd).cpu().numpy()
    n = int((Y.view(np.uint32) != ref.view(np.uint32)).sum())
    bad += n > 0
    rows = np.nonzero((Y.view(np.uint32) != ref.view(np.uint32)).any(axis=1))[0]
    cols = np.nonzero((Y.view(np.uint32) != ref.view(np.uint32)).any(axis=0))[0]
    print(f"run {r}: {n} values differ; rows {rows[:12].tolist()}{'...' if len(rows) > 12 else ''} ({len(rows)}), "
          f"cols {len(cols)}", flush=True)
enc.close()
print(f"{bad} of {reps} runs differ from the oracle")
sys.exit(1 if bad else 0)
