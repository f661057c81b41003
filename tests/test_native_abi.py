"""CPU checks of the drop-in boundary: libdclip.so loads, exports every entry point declared
in include/dclip.h, and rejects bad arguments with an error message (argument validation
runs before any HIP call, so these run without a GPU)."""
import ctypes
import os
import re

import pytest

from helpers import ROOT
from denseclip_vit_multimodal_amd import _native as N


def declared_symbols():
    with open(os.path.join(ROOT, "include", "dclip.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(dclip_\w+)\s*\(", src, re.M)))


def test_header_and_binding_agree():
    assert declared_symbols() == N.EXPORTED


def test_library_exports_every_declared_symbol():
    lib = N.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.dclip_abi_version() == 7


def test_no_oracle_in_product_package():
    pkg = os.path.join(ROOT, "denseclip_vit_multimodal_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".hip", ".h", ".cpp")):
                with open(os.path.join(dirpath, fn)) as f:
                    txt = f.read()
                assert "oracle" not in txt.replace("no oracle", ""), fn


@pytest.mark.parametrize("call,needle", [
    (lambda L: L.dclip_gemm(0, 0, None, 64, None, 64, 64, 64, 64, 1, 1.0, None, None, None, 0, 0, None, 0, 64, None, 0, None),
     "f16/bf16"),
    (lambda L: L.dclip_gemm(0, 2, None, 64, None, 64, 64, 64, 100, 1, 1.0, None, None, None, 0, 0, None, 2, 64, None, 0, None),
     "multiple of 64"),
    (lambda L: L.dclip_gemm(4, 2, None, 64, None, 64, 64, 64, 64, 2, 1.0, None, None, None, 0, 0, None, 0, 64, None, 0, None),
     "multiple of 64*splits"),
    (lambda L: L.dclip_attn_fwd(2, None, None, None, 1, 8, 2, 32, 1.0, None), "head_dim must be 64"),
    (lambda L: L.dclip_layernorm_fwd(None, 0, None, None, None, 0, None, None, 4, 4098, 1e-5, None), "cols"),
    (lambda L: L.dclip_score_map(None, 2, 0, 0, 512, None, None, 1, 4, 512, 40, 1e-12, None), "K must be"),
    (lambda L: L.dclip_row_mean(None, 2, 0, 0, 100, 1, 4, 100, None, None, None), "C % 8"),
    (lambda L: L.dclip_im2col(None, 0, None, 0, 768, 1, 3, 8, 8, 16, None), "smaller than one patch"),
])
def test_argument_errors_are_reported(call, needle):
    L = N.load()
    rc = call(L)
    assert rc == -1
    assert needle in L.dclip_last_error().decode()


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(N.NativeError):
        N.load(str(tmp_path / "nope.so"))


def test_dclip_lib_mismatch_raises(tmp_path):
    """DCLIP_LIB pointing at another libdclip.so than the one libdclip_torch.so binds
    (its own directory) raises instead of configuring a library no op calls."""
    import subprocess
    import sys
    other = tmp_path / "libdclip.so"
    other.write_bytes(b"")
    code = "from denseclip_vit_multimodal_amd import _torch_ops; _torch_ops.load()"
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       env=dict(os.environ, DCLIP_LIB=str(other)), timeout=300)
    assert r.returncode != 0 and "DCLIP_LIB" in r.stderr, r.stderr[-2000:]
