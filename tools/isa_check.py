"""Instruction audit of a built gfx950 object: which kernels contain given mnemonics.

Used by the Makefile (after pg_dense_bwd.o is built) and by tests/test_host.py: the bf16 input-gradient kernels gave
timing-dependent gate gradients when the SLP vectoriser put packed-FP32 VALU ops (v_pk_fma_f32 / v_pk_mul_f32) next
to their v_mfma_f32_32x32x16_bf16 products ("Reproducibility"); pg_dense_bwd.hip is built with
-fno-slp-vectorize, and this check fails the build if a compiler change brings such ops back into a dgrad kernel.

    python tools/isa_check.py build/pg_dense_bwd.o            # exit 1 if a dgrad kernel holds packed-FP32 ops
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
PACKED_FP32 = ("v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32")


def disassemble(obj: str) -> str:
    """The gfx950 device code of a hipcc -c object, disassembled."""
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fatbin"), os.path.join(d, "dev.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "o")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--targets={TARGET}", f"--input={fb}",
                        f"--output={co}", "--unbundle"], check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True,
                              text=True).stdout


def kernel_mnemonics(obj: str, kernel_re: str, mnemonics=PACKED_FP32) -> dict:
    """{kernel symbol: number of instructions among `mnemonics`} for the kernels whose symbol matches kernel_re."""
    out: dict = {}
    cur = None
    head = re.compile(r"^[0-9a-f]+ <(.+)>:$")
    for line in disassemble(obj).splitlines():
        m = head.match(line)
        if m:
            cur = m.group(1) if re.search(kernel_re, m.group(1)) else None
            if cur is not None:
                out.setdefault(cur, 0)
            continue
        if cur is not None:
            tok = line.strip().split()
            if tok and tok[0] in mnemonics:
                out[cur] += 1
    return out


def main(argv) -> int:
    obj = argv[1] if len(argv) > 1 else "build/pg_dense_bwd.o"
    found = kernel_mnemonics(obj, r"dgrad")
    if not found:
        print(f"isa_check: no dgrad kernel found in {obj}", file=sys.stderr)
        return 1
    bad = {k: v for k, v in found.items() if v}
    if bad:
        print(f"isa_check: packed-FP32 VALU ops in dgrad kernels of {obj}: {bad}", file=sys.stderr)
        return 1
    print(f"isa_check: {len(found)} dgrad kernels, no packed-FP32 VALU ops")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
