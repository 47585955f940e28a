"""Per-kernel register / scratch / LDS use of the built library's gfx950 code object.

    python scripts/kernel_resources.py [lib.so] [name-substring ...]

Reads the clang offload bundle inside the .hip_fatbin section (no GPU needed), writes the
gfx950 code object to /tmp and prints llvm-readelf's AMDHSA metadata per kernel: VGPRs, AGPRs,
SGPRs, scratch bytes a lane (spills), LDS bytes.  Used to check that no hot kernel spills."""
import os
import re
import struct
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/llvm/bin/llvm-readelf"


def code_object(lib):
    data = open(lib, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = data.find(magic)
    if pos < 0:
        raise SystemExit("no offload bundle in " + lib)
    n = struct.unpack_from("<Q", data, pos + 24)[0]
    p = pos + 32
    for _ in range(n):
        off, size, idl = struct.unpack_from("<QQQ", data, p)
        ident = data[p + 24:p + 24 + idl].decode()
        p += 24 + idl
        if "gfx950" in ident:
            return data[pos + off:pos + off + size]
    raise SystemExit("no gfx950 code object")


def kernels(lib):
    co = code_object(lib)
    path = "/tmp/lrs_gfx950.co"
    with open(path, "wb") as f:
        f.write(co)
    txt = subprocess.run([READELF, "--notes", path], capture_output=True, text=True).stdout
    out = []
    for blk in re.split(r"\n  - \.agpr_count:", txt)[1:]:
        def get(k):
            m = re.search(r"\n    \.%s:\s+(\S+)" % k, blk)
            return m.group(1) if m else "-1"
        out.append({"name": get("name"), "vgpr": int(get("vgpr_count")), "agpr": int(blk.split()[0]),
                    "sgpr": int(get("sgpr_count")), "scratch": int(get("private_segment_fixed_size")),
                    "lds": int(get("group_segment_fixed_size"))})
    return out


def main():
    args = sys.argv[1:]
    lib = args.pop(0) if args and args[0].endswith(".so") else os.path.join(ROOT, "ltr-lowrank-sdp_amd", "_build",
                                                                           "liblrsdp.so")
    ks = kernels(lib)
    names = subprocess.run(["c++filt"], input="\n".join(k["name"] for k in ks), capture_output=True,
                           text=True).stdout.split("\n")
    for k, dn in zip(ks, names):
        dn = dn.split("(")[0]
        if args and not any(a in dn for a in args):
            continue
        flag = "  SPILLS" if k["scratch"] > 0 else ""
        print(f"{dn:60s} vgpr {k['vgpr']:3d} agpr {k['agpr']:3d} sgpr {k['sgpr']:3d} scratch {k['scratch']:4d} "
              f"lds {k['lds']:6d}{flag}")


if __name__ == "__main__":
    main()
