"""Generate the golden fixtures under tests/golden/.

Two kinds of fixture, kept apart on purpose:

1. ``kat.json`` -- known-answer tests whose EXPECTED values do not come from our oracle:
   KAT-1 is the reference's own fixture (inputs of /root/reference/src/test_quantize.cu:38-62,
   range 127 at :76) with the outputs SURVEY.md s4 records from the survey's probe that ran the
   reference's own __host__ __device__ functors over the reference kernels' loop structure
   (before this build existed).  The reference itself cannot be compiled here (it needs
   cuda_runtime.h / curand.h), so this is the strongest pin available.  KAT-2 is the absmax
   seeding quirk of op_reduction.cuh:80/105 from the same source.  The values below are typed in
   from SURVEY.md, not computed.

2. ``cases.npz`` -- regression fixtures produced by the CPU oracle (oracle/qgemm_oracle.c) on
   seeded and hand-made edge-case inputs: random U(-1,1) shapes, ragged shapes, K = 1, M = 1,
   zero rows/columns, the absmax quirk with and without int8 overflow, NaN and inf inputs.
   They freeze the oracle's answers (so a later edit of the restatement cannot drift silently) and
   give the GPU tests exact expected bits.  128^3 cases store SHA-256 digests instead of arrays.

Run from the repo root:  python tests/golden/gen_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import oracle as O  # noqa: E402

KAT = {
    "source": "SURVEY.md s4 (KAT table): reference fixture test_quantize.cu:38-62, outputs from the "
              "survey probe of the reference's own functors (op_reduction.cuh:7-25, op_elemwise.cuh:93-143)",
    "kat1": {
        "X": [[2, -1, -1], [0, 3, 2], [-1, -1, 0]],
        "W": [[-1, 0], [0, -2], [-1, 2]],
        "range": 127.0,
        "Cx": [2.0, 3.0, 1.0],
        "Cw": [1.0, 2.0],
        "Xq": [[127, -63, -63], [0, 127, 84], [-127, -127, 0]],
        "Acc": [[-8128, 0], [-10668, -5461], [16129, 16129]],
        "O_bits": ["0xbf810204", "0x00000000", "0xbffdfbf8", "0xc0020408", "0x3f800000", "0x40000000"],
        "unquantized": [[-1, 0], [-2, -2], [1, 2]],
        "printed_signed_mean": 0.003937006,
    },
    "kat2": {"row": [-0.9, 0.5, -0.3, 0.8], "absmax": 0.8},
}


def _digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def edge_cases():
    """(name, X, W) hand-made inputs that exercise the reference's corner semantics."""
    rng = np.random.default_rng(1234)
    cases = []
    # absmax quirk: negative first element has the largest magnitude (scale = 2nd largest)
    X = rng.uniform(-1, 1, (8, 40)).astype(np.float32)
    W = rng.uniform(-1, 1, (40, 9)).astype(np.float32)
    X[0, 0] = -0.99
    X[0, 1:] = np.clip(X[0, 1:], -0.9, 0.9)
    W[0, 3] = -0.995
    W[1:, 3] = np.clip(W[1:, 3], -0.6, 0.6)
    cases.append(("quirk_no_overflow", X, W))
    # quirk with int8 overflow: x0 = -1, the rest <= 0.5 -> x0*sx = -254 (saturates to -128)
    X = rng.uniform(-0.5, 0.5, (5, 33)).astype(np.float32)
    W = rng.uniform(-0.25, 0.25, (33, 7)).astype(np.float32)
    X[2, 0] = -1.0
    W[0, 5] = -1.0
    cases.append(("quirk_overflow", X, W))
    # zero row in X, zero column in W, negative-zero seed
    X = rng.uniform(-1, 1, (6, 20)).astype(np.float32)
    W = rng.uniform(-1, 1, (20, 5)).astype(np.float32)
    X[1, :] = 0.0
    X[3, :] = 0.0
    X[3, 0] = -0.0
    W[:, 2] = 0.0
    cases.append(("zero_row_col", X, W))
    # NaN at k >= 1 is skipped by AbsMaxFunc; a NaN seed sticks; inf inputs
    X = rng.uniform(-1, 1, (6, 24)).astype(np.float32)
    W = rng.uniform(-1, 1, (24, 6)).astype(np.float32)
    X[0, 5] = np.nan
    X[2, 0] = np.nan
    X[4, 7] = np.inf
    W[3, 1] = -np.inf
    W[0, 4] = np.nan
    cases.append(("nan_inf", X, W))
    # K = 1 (reference UB for W; defined here as the per-column seed), M = 1, N = 1
    cases.append(("k1", rng.uniform(-1, 1, (7, 1)).astype(np.float32), rng.uniform(-1, 1, (1, 5)).astype(np.float32)))
    cases.append(("m1_decode", rng.uniform(-1, 1, (1, 300)).astype(np.float32),
                  rng.uniform(-1, 1, (300, 70)).astype(np.float32)))
    cases.append(("n1", rng.uniform(-1, 1, (9, 50)).astype(np.float32), rng.uniform(-1, 1, (50, 1)).astype(np.float32)))
    # large magnitudes and subnormals
    X = (rng.uniform(-1, 1, (4, 16)) * 3e30).astype(np.float32)
    W = (rng.uniform(-1, 1, (16, 4)) * 1e-40).astype(np.float32)
    cases.append(("extreme_magnitudes", X, W))
    return cases


def seeded_cases():
    """(name, M, N, K, seed) on the shared generator (oracle.inputs: X seed 2s, W seed 2s+1)."""
    out = [(f"u128_s{s}", 128, 128, 128, s) for s in (1, 2, 3, 4)]
    out += [("ragged_67x45x131", 67, 45, 131, 5), ("ragged_33x257x129", 33, 257, 129, 6),
            ("tile_256x256x128", 256, 256, 128, 7), ("ragged_257x255x129", 257, 255, 129, 8),
            ("ragged_300x1x7", 300, 1, 7, 9), ("small_3x2x3_rand", 3, 2, 3, 10)]
    return out


def main():
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(KAT, f, indent=1)

    arrays = {}
    index = []
    for name, X, W in edge_cases():
        Ov, d = O.quantized_mm(X, W, intermediates=True)
        arrays[f"{name}/X"], arrays[f"{name}/W"] = X, W
        arrays[f"{name}/O"], arrays[f"{name}/Cx"], arrays[f"{name}/Cw"] = Ov, d["Cx"], d["Cw"]
        arrays[f"{name}/Xq"], arrays[f"{name}/Wq"], arrays[f"{name}/Acc"] = d["Xq"], d["Wq"], d["Acc"]
        index.append(dict(name=name, kind="explicit", M=X.shape[0], N=W.shape[1], K=X.shape[1]))
    for name, M, N, K, seed in seeded_cases():
        X, W = O.inputs(M, N, K, seed)
        Ov, d = O.quantized_mm(X, W, intermediates=True)
        C = O.mm_fp32(X, W)
        rec = dict(name=name, kind="seeded", M=M, N=N, K=K, seed=seed,
                   x_head=X.ravel()[:8].tolist(), w_head=W.ravel()[:8].tolist(),
                   O_sha256=_digest(Ov), Acc_sha256=_digest(d["Acc"]), Xq_sha256=_digest(d["Xq"]),
                   Wq_sha256=_digest(d["Wq"]), Cx_sha256=_digest(d["Cx"]), Cw_sha256=_digest(d["Cw"]),
                   C_sha256=_digest(C), signed_mean=O.signed_mean_error(C, Ov))
        if M * N <= 5000:
            arrays[f"{name}/O"] = Ov
        index.append(rec)
    np.savez_compressed(os.path.join(HERE, "cases.npz"), **arrays)
    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump(index, f, indent=1)
    print(f"wrote {len(index)} cases")


if __name__ == "__main__":
    main()
