"""bench.py's roofline bookkeeping from the committed rocprof leg summaries (CPU only): the newest
profiles/<tag>_<leg>_pmc.json is picked by name, each stage gets its counter traffic and rocprof
time, and the stage labels name the kernels the profile saw (k_bw_b for the bandwidth regime's
fused stage B, not the k_it_b the kernel-path table would guess)."""
import glob
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    argv = sys.argv
    sys.argv = ["bench.py"]
    try:
        spec.loader.exec_module(mod)
    finally:
        sys.argv = argv
    return mod


def test_leg_profile_newest_and_labels():
    b = _bench()
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_g81_pmc.json")))
    assert files, "no committed g81 leg profile"
    prof = b.leg_profile("g81")
    assert prof["_source"].endswith(os.path.basename(files[-1]).replace("_pmc.json", "_summary.md"))
    res = {"kernel": "B: k_it_b (line search)", "a_uut": {},
           "stages": [{"stage": "A: k_it_a (control)", "kernel": "k_it_a"},
                      {"stage": "B: k_it_b (line search)", "kernel": "k_it_b"}]}
    out = b.attach_traffic(res, "g81")
    seen = {v["stage"]: [] for k, v in prof.items() if not k.startswith("_")}
    for k, v in prof.items():
        if not k.startswith("_"):
            seen[v["stage"]].append(k.split("::")[-1].split("<")[0])
    for o in out["stages"]:
        st = o["stage"][0]
        assert o["kernel"] == " + ".join(dict.fromkeys(seen[st])), (o, seen)
        assert o["traffic"] == prof["_stages"][st]["traffic_bytes"]
        assert o["rocprof_us"] == prof["_stages"][st]["rocprof_us"]
    assert out["kernel"].startswith("B: ") and out["kernel"].split(" (")[0][3:] == out["stages"][1]["kernel"]
    assert out["traffic"] == prof["_stages"]["B"]["traffic_bytes"]
    assert "summary.md" in out["traffic_source"]
