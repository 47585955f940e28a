"""GPU box: which of the restructured bandwidth-regime kernels changes bits -- K trips on the
bandwidth path under each LRS_BW_A / LRS_BW_B / LRS_A1_PRE setting (one subprocess each), max
|diff| per array against all three off."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_bw_kernels import run  # noqa: E402
from golden_util import instance  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "mc_torus12x10"
src = name if name.startswith("rsp:") else instance(name)
K = int(sys.argv[2]) if len(sys.argv) > 2 else 1
off = {"LRS_BW_A": "0", "LRS_BW_B": "0", "LRS_A1_PRE": "0"}
base = run(src, K, "/tmp/bw_base.npz", off)
for on in ("LRS_BW_A", "LRS_BW_B", "LRS_A1_PRE"):
    env = dict(off)
    env[on] = "1"
    o = run(src, K, "/tmp/bw_one.npz", env)
    d = {k: float(np.max(np.abs(o[k] - base[k]))) for k in ("R", "G", "cvs", "lam", "s", "y", "tau", "D")}
    print(name, "K", K, on, d, flush=True)
