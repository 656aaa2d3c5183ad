#!/usr/bin/env python3
"""VGPR / AGPR / SGPR / scratch / LDS of every gfx950 kernel in a hipcc object or shared library.

    python scripts/kernel_resources.py build/obj/k_conv_tile.o [--grep conv_tile]

Extracts the device code object with clang-offload-bundler (objects) or from the .hip_fatbin
section (shared libraries) and reads the AMDGPU metadata notes with llvm-readelf.
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(path: str, tmp: str) -> str:
    out = os.path.join(tmp, "dev.co")
    fb = os.path.join(tmp, "fatbin.bin")
    r = subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", path, os.path.join(tmp, "x.o")],
                       capture_output=True, text=True)
    if r.returncode != 0:
        sys.exit(r.stderr)
    r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle", f"--input={fb}",
                        f"--output={out}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], capture_output=True, text=True)
    if r.returncode != 0:
        sys.exit(r.stderr)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("obj")
    ap.add_argument("--grep", default="")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        co = code_object(a.obj, tmp)
        txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    rows, cur = [], {}
    for ln in txt.splitlines():
        m = re.match(r"\s+- \.agpr_count:\s+(\d+)", ln)
        if m:
            if cur:
                rows.append(cur)
            cur = {"agpr": int(m.group(1))}
            continue
        for key, field in ((".name:", "name"), (".vgpr_count:", "vgpr"), (".sgpr_count:", "sgpr"),
                           (".private_segment_fixed_size:", "scratch"), (".group_segment_fixed_size:", "lds"),
                           (".vgpr_spill_count:", "vspill")):
            m = re.match(r"\s+" + re.escape(key) + r"\s+(\S+)", ln)
            if m and cur is not None:
                v = m.group(1)
                cur[field] = int(v) if v.isdigit() else v
    if cur:
        rows.append(cur)
    for r in rows:
        if a.grep and a.grep not in str(r.get("name", "")):
            continue
        print(f"{r.get('vgpr', '?'):>4} v {r.get('agpr', '?'):>4} a {r.get('sgpr', '?'):>4} s "
              f"scratch {r.get('scratch', '?'):>5} spill {r.get('vspill', '?'):>4}  {r.get('name')}")


if __name__ == "__main__":
    main()
