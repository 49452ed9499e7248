"""CPU checks of the boundary: libslx_hip.so loads and exports every entry point include/slx.h declares,
and the ctypes descriptors match the C struct layouts (no compute without a GPU)."""
import ctypes
import os
import re

import pytest

from simlingo_amd import kernels as K
from simlingo_amd.decode import DecGemvDesc
from simlingo_amd.frames import FrameDesc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "slx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(slx_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_header_symbol():
    lib = K.lib()
    names = header_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_bindings_cover_header():
    bound = set(K.exported_symbols())
    unbound = [n for n in header_functions() if n not in bound]
    assert not unbound, unbound


def test_abi_version_and_error_path():
    assert K.lib().slx_abi_version() == 1
    # argument validation runs on the host and must fail loudly without touching a GPU
    d = K.GemmDesc()
    d.layout, d.M, d.N, d.K, d.batch, d.lda, d.ldb = 0, 8, 8, 7, 1, 8, 8
    rc = K.lib().slx_gemm_bf16(ctypes.byref(d), None)
    assert rc == -22
    assert b"multiple of 8" in K.lib().slx_last_error()
    with pytest.raises(RuntimeError, match="slx_attn_fwd"):
        a = K.AttnDesc()
        a.head_dim = 128
        K.check(K.lib().slx_attn_fwd(ctypes.byref(a), None), "slx_attn_fwd")


def test_struct_layouts_match_header(tmp_path):
    """Compile a probe against include/slx.h with gcc and compare sizeof/offsetof with the ctypes mirrors."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    structs = {"slx_gemm_desc": K.GemmDesc, "slx_gemm_lt_desc": K.GemmLtDesc, "slx_attn_desc": K.AttnDesc,
               "slx_attn_bwd_desc": K.AttnBwdDesc,
               "slx_norm_desc": K.NormDesc, "slx_sgemm_desc": K.SgemmDesc,
               "slx_lora_down_desc": K.LoraDownDesc,
               "slx_lora_bwd_desc": K.LoraBwdDesc, "slx_dropout_bits_desc": K.DropoutBitsDesc,
               "slx_dropout_bits_job": K.DropoutBitsJob, "slx_dec_gemv_desc": DecGemvDesc,
               "slx_lora_grad_job": K.LoraGradJob,
               "slx_frame_desc": FrameDesc}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "slx.h"', "int main(void){"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    for line in filter(None, out):
        cname, field, val = line.split()
        cls = structs[cname]
        want = ctypes.sizeof(cls) if field == "size" else getattr(cls, field).offset
        assert int(val) == want, (cname, field, val, want)
