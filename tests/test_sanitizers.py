"""Host-code sanitizers: the native runtime under ASan + UBSan.

The C++ sampler / voxel generator / binvox IO are rebuilt with
``-fsanitize=address,undefined`` and exercised in a fresh interpreter with the
ASan runtime preloaded; any heap overflow, use-after-free or UB aborts it.
(GPU sanitizers are not used: host code only.)
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import _rt
assert _rt.__file__.startswith(sys.argv[1]), _rt.__file__
clauses = [[1], [-2, 3], [2, 4, -5], [-3, -4], [5, 6, 7], [-6, -7], [1, -8]]
r = _rt.sample_diverse(9, clauses, 12, 50.0, 3, 0, True)
assert len(r["products"]) == 12 and all(_rt.check(9, clauses, p) for p in r["products"])
_rt.jaccard_matrix(r["products"], 9)
_rt.random_products(9, clauses, 5, 1)
bits, lab = _rt.generate_voxels(24, 32, 1, threads=4)
v = _rt.unpack_bits(bits, bits.size * 8)
assert (_rt.pack_bits(v) == bits.reshape(-1)).all()
g = (np.random.default_rng(0).random((16, 16, 16)) < 0.4).astype(np.uint8)
_rt.write_binvox(sys.argv[2], g, [0.0, 0.0, 0.0], 1.0)
back, _, _ = _rt.read_binvox(sys.argv[2])
assert (back == g).all()
print("sanitized runtime ok")
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_runtime_under_asan_ubsan(tmp_path):
    from featurenet_amd import _build

    so = _build.build_runtime_sanitized(tmp_path / "asan")
    libasan = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isfile(libasan):
        pytest.skip("libasan not available")
    env = dict(os.environ, LD_PRELOAD=libasan, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-c", DRIVER, str(so.parent), str(tmp_path / "t.binvox")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "sanitized runtime ok" in r.stdout
