"""Static guard on the inline-asm transposing LDS reads (csrc/include/ddpx_pipe.h ``frag_tr``/``frag_settle``).

The compiler's waitcnt pass cannot see ``ds_read_b64_tr_b16`` issued from inline asm, so the kernels rely on
``frag_settle`` redefining both halves of every fragment in the asm statement that waits.  This disassembles
the gfx950 code objects of the built kernel library (the binary that ships to the GPU) and checks that no
instruction touches a transposing read's destination registers before its ``s_waitcnt lgkmcnt(0)``.
"""
import glob
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LLVM = "/opt/rocm/lib/llvm/bin"


def test_no_reads_of_pending_transposed_fragments(tmp_path):
    if not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("ROCm llvm-objdump not available")
    from ddpx.runtime import build
    libs = build.build()
    lib = str(tmp_path / "libddpx_kernels.so")
    shutil.copy(libs["kernels"], lib)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", lib], check=True, capture_output=True)
    objs = sorted(glob.glob(lib + ".*gfx950"))
    assert objs, "no gfx950 code objects in the kernel library"
    import check_tr_reads
    checked = 0
    for o in objs:
        dis = o + ".s"
        with open(dis, "w") as f:
            subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", o], check=True, stdout=f)
        assert check_tr_reads.main(dis) == 0, o
        checked += sum(1 for ln in open(dis) if "ds_read_b64_tr_b16" in ln)
    assert checked > 0, "no transposing reads found: is the GEMM core still built?"
