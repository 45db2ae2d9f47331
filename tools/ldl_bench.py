"""Dense LDL' of the coupled-hands Hessian block: the kernel's register method against a
16-column-panel factor with MFMA trailing updates (tools/ldl_bench.hip), cycles per factor of
one wave at block sizes 16 / 28 / 40 / 52, and the factor's accuracy (max |L D L' - A| / max |A|).
Run on the GPU box: python tools/ldl_bench.py  (tools/libldlbench.so built beforehand)."""
import ctypes as C
import json
from pathlib import Path

import numpy as np
import torch

lib = C.CDLL(str(Path(__file__).resolve().parent / "libldlbench.so"))
lib.ldl_bench_run.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]


def spd(n, nmat, rng):
    """Newton-Hessian-like blocks: M-like SPD part plus contact rows J' D J."""
    out = np.empty((nmat, n, n), np.float32)
    for i in range(nmat):
        G = rng.normal(size=(n, n)) / np.sqrt(n)
        J = rng.normal(size=(3 * max(1, n // 8), n))
        A = G @ G.T + np.diag(rng.uniform(0.05, 1.0, n)) + J.T @ np.diag(rng.uniform(0, 50, len(J))) @ J
        out[i] = A
    return out


rng = np.random.RandomState(0)
NMAT = 512
for n in (16, 28, 40, 52):
    A = spd(n, NMAT, rng)
    dA = torch.from_numpy(A).cuda()
    res = {"n": n}
    for m, name in ((0, "reg"), (1, "mfma")):
        out = torch.zeros_like(dA)
        cyc = torch.zeros(NMAT, dtype=torch.int64, device="cuda")
        assert lib.ldl_bench_run(m, n, dA.data_ptr(), out.data_ptr(), cyc.data_ptr(), NMAT, 20) == 0
        err = (out.cpu().numpy() - A).reshape(NMAT, -1)
        rel = np.abs(err).max(axis=1) / np.abs(A.reshape(NMAT, -1)).max(axis=1)
        c = cyc.cpu().numpy()
        res[name] = {"cycles_median": float(np.median(c)), "cycles_p90": float(np.percentile(c, 90)),
                     "rel_err_max": float(rel.max())}
    print(json.dumps(res), flush=True)
