"""Writes the build provenance of the in-tree libraries as JSON (Makefile target
build_info.json): source commit + dirty flag, hipcc version, compile flags, SHA-256 and size
of each shipped .so, and the build time.  usage: python3 build_info.py <lib dir> "<flags>"."""
import datetime
import hashlib
import json
import os
import subprocess
import sys


def run(cmd):
    try:
        return subprocess.run(cmd, capture_output=True, text=True, check=False).stdout.strip()
    except OSError:
        return ""


def main():
    out, flags = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    here = os.path.dirname(os.path.abspath(__file__))
    git = ["git", "-C", here]
    libs = {}
    for name in ("libeverest_amd.so", "libeverest_amd_torch.so"):
        path = os.path.join(out, name)
        if os.path.exists(path):
            with open(path, "rb") as f:
                libs[name] = {"sha256": hashlib.sha256(f.read()).hexdigest(), "bytes": os.path.getsize(path)}
    hip = run(["/opt/rocm/bin/hipcc", "--version"]).splitlines()
    info = {
        "commit": run(git + ["rev-parse", "--short=12", "HEAD"]),
        "dirty": bool(run(git + ["status", "--porcelain", "--", "."])),
        "compiler": next((line for line in hip if "clang version" in line or "HIP version" in line), ""),
        "flags": flags,
        "libs": libs,
        "built_utc": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
        "command": "make -C everest_amd/csrc ARCH=gfx950 (__graft_entry__.build())",
    }
    print(json.dumps(info, indent=1))


if __name__ == "__main__":
    main()
