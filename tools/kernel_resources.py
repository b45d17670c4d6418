"""Per-kernel resources of the built gfx950 library: VGPRs, SGPRs, LDS, scratch (private
segment) bytes per lane, read from the AMDGPU code-object metadata in the library's
.hip_fatbin section (clang offload bundles -> llvm-readelf --notes).

A kernel with private_segment_fixed_size > 0 spills registers (or keeps a dynamically
indexed private array) in scratch memory: every lane's spill traffic goes through L2 / HBM
(hvi_kdb<5> wrote ~58 MB of scratch per launch before round 4 — its WRITE_SIZE counter).
tests/test_native_cpu.py asserts the evaluation chain's kernels stay at zero.

usage: python tools/kernel_resources.py [lib.so] [--scratch-only]   (one JSON object per line)"""
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib: str, arch: str = "gfx950"):
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", lib,
                        os.path.join(td, "stripped.so")], check=True, capture_output=True)
        data = open(fb, "rb").read()
    pos = 0
    while True:
        j = data.find(MAGIC, pos)
        if j < 0:
            break
        ne = struct.unpack_from("<Q", data, j + 24)[0]
        p = j + 32
        for _ in range(ne):
            off, size, il = struct.unpack_from("<QQQ", data, p)
            p += 24
            tid = data[p:p + il].decode(errors="replace")
            p += il
            if arch in tid:
                yield data[j + off:j + off + size]
        pos = j + 1


def kernels(lib: str):
    """{kernel symbol: {vgpr, sgpr, lds, scratch}} over every gfx950 code object."""
    out = {}
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".o") as f:
            f.write(co)
            f.flush()
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name], check=True,
                                   capture_output=True, text=True).stdout
        # one kernel's fields are one YAML list entry ("  - .agpr_count: ..." opens it); its
        # .name sits in the middle of the alphabetical field order, so collect the entry first
        cur = None
        for line in notes.splitlines():
            m = re.match(r"(\s*)(- )?\.(\w+):\s+(\S+)", line)
            if not m:
                continue
            ind, item, k, v = m.groups()
            if item and len(ind) <= 4:
                cur = {}
            if cur is None:
                continue
            if k == "name" and not v.endswith(".kd"):
                out[v] = cur
            elif k in ("vgpr_count", "sgpr_count", "group_segment_fixed_size", "private_segment_fixed_size",
                       "agpr_count", "max_flat_workgroup_size"):
                key = {"group_segment_fixed_size": "lds", "private_segment_fixed_size": "scratch",
                       "max_flat_workgroup_size": "wg"}.get(k, k)
                cur[key] = int(v)
    return out


def occupancy(r: dict, lds_dyn: int = 0) -> dict:
    """Resident workgroups per CU of a kernel at its maximum workgroup size: the unified
    VGPR + AGPR file (512 per SIMD lane, granule 8), 160 KB of LDS per CU (plus dynamic LDS
    the launch adds), at most 8 waves per SIMD...  {wgs_per_cu, waves_per_simd, limit}."""
    wg = r.get("wg", 256)
    wpw = max(1, -(-wg // 64))                 # waves per workgroup
    regs = -(-(r.get("vgpr_count", 0) + r.get("agpr_count", 0)) // 8) * 8
    by_regs = (512 // regs if regs else 8) * 4 // wpw
    lds = r.get("lds", 0) + lds_dyn
    by_lds = 160 * 1024 // lds if lds else 64
    by_waves = 8 * 4 // wpw
    n = min(by_regs, by_lds, by_waves)
    lim = "regs" if n == by_regs else ("lds" if n == by_lds else "waves")
    return {"wgs_per_cu": n, "waves_per_simd": n * wpw / 4, "limit": lim}


def demangle(names):
    for tool in (os.path.join(LLVM, "llvm-cxxfilt"), "c++filt"):
        try:
            r = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True)
        except OSError:
            continue
        if r.returncode == 0:
            return r.stdout.splitlines()
    return list(names)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args else os.path.join(ROOT, "everest_amd", "_lib", "libeverest_amd.so")
    ks = kernels(lib)
    names = sorted(ks)
    for raw, pretty in zip(names, demangle(names)):
        r = ks[raw]
        if "--scratch-only" in sys.argv and not r.get("scratch"):
            continue
        print(json.dumps({"kernel": pretty, **r, **occupancy(r)}))


if __name__ == "__main__":
    main()
