"""CPU checks of the BASELINE config fixtures the GPU tests read (tests/test_gpu_configs.py):
the reference's own solves (solves_configs.json, scripts/make_golden_configs.py) and its final
theta iterates (configs_final_*.npz, scripts/make_golden_configs_final.py) match the instances
the seeded generators write and the trace blocks the certified-interval test relies on."""
import hashlib
import importlib
import json
import os

import numpy as np

from golden_util import GOLDEN, block_traces


def test_theta_final_iterates_fit_their_instances(tmp_path):
    inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
    gold = {g["config"]: g for g in json.load(open(os.path.join(GOLDEN, "solves_configs.json")))}
    for name, K in (("theta3", 1), ("theta3x3", 3)):
        path = inst.config_instance(name, str(tmp_path))
        assert hashlib.sha256(open(path, "rb").read()).hexdigest() == gold[name]["sha256"]
        tr = block_traces(path)
        assert tr == [1.0] * K
        z = np.load(os.path.join(GOLDEN, f"configs_final_{name}.npz"))
        assert z["ranks"].shape == (K,)
        assert z["R"].size == 150 * int(z["ranks"].sum())
        assert z["lam"].size == int(z["m"]) and np.isfinite(z["lam"]).all() and np.isfinite(z["R"]).all()
        # the final iterate's trace per block: the reference stops near tr X_k = 1
        R = z["R"]
        off = 0
        for r in z["ranks"]:
            blk = R[off:off + 150 * int(r)]
            assert abs(float(blk @ blk) - 1.0) < 1e-3
            off += 150 * int(r)
