"""The engine's variation pow (csrc/detmath.h det_pow, exported for the host as mv_det_pow)
against its oracle restatement (oracle/device_order.py:det_pow): bit-identical on the
argument ranges of polynomial mutation (softmax_mutation.py:77-103: x^(eta+1) with x in
[0, 1], val^(1/(eta+1)) with val in [0, 2]) and of the SBX option (beta^-(eta+1),
u^(1/(eta+1))), plus the special values; and within 1 ulp of np.power (the reference's pow)
there.  No GPU needed: the host build of detmath.h is the same IEEE operation sequence as
the device build (tests/test_gpu_parity.py::test_variation_vs_oracle checks the device)."""
import os

import numpy as np
import pytest

from oracle.device_order import det_pow


def _cases():
    rng = np.random.default_rng(0)
    n = 200_000
    yield "pm x^21", rng.random(n), 21.0
    yield "pm val^(1/21)", rng.random(n) * 2.0, 1.0 / 21.0
    yield "pm tiny val", np.exp(rng.uniform(-700.0, 0.0, n)), 1.0 / 21.0
    yield "sbx beta^-31", 1.0 + np.exp(rng.uniform(-30.0, 10.0, n)), -31.0
    yield "sbx u^(1/31)", rng.random(n) * 2.0, 1.0 / 31.0


def _lib_pow():
    from moeva2_amd import _native

    try:
        _native.lib()
    except _native.NativeError as e:  # pragma: no cover
        pytest.skip(str(e))
    return _native.det_pow


@pytest.mark.parametrize("name,x,y", list(_cases()), ids=[c[0] for c in _cases()])
def test_det_pow_host_build_matches_oracle_and_np_power(name, x, y):
    host = _lib_pow()
    got = host(x, y)
    ref = det_pow(x, y)
    assert np.array_equal(got.view(np.int64), ref.view(np.int64)), name
    npw = np.power(x, y)
    ok = np.isfinite(npw) & (np.abs(npw) > 1e-300)
    ulp = np.abs(got[ok] - npw[ok]) / np.spacing(np.abs(npw[ok]))
    assert ulp.max() <= 1.0, (name, ulp.max())


def test_det_pow_special_values():
    host = _lib_pow()
    x = np.array([0.0, 1.0, np.inf, -1.0, np.nan, 2.0, 0.5, 1e-310, 5e-324, 1e300])
    for y in (21.0, 1.0 / 21.0, -31.0, 0.0, np.nan, 2.5):
        a, b = host(x, np.full_like(x, y)), det_pow(x, y)
        assert np.array_equal(a, b, equal_nan=True), y
    assert det_pow(0.0, 21.0) == 0.0 and np.isnan(det_pow(1.0, np.nan))  # NaN first
    assert det_pow(0.25, 0.5) == 0.5 and det_pow(3.0, 4.0) == 81.0


def test_det_pow_fma_products_bit_identical(tmp_path):
    """The device calls det_pow<true>: exact products from an FMA instead of Dekker's split
    (csrc/detmath.h).  Built for the host and run on 3 M SBX / mutation arguments, it
    returns det_pow<>'s bits -- the oracle's -- on every one."""
    import shutil
    import subprocess

    cxx = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(cxx):
        pytest.skip("hipcc not found")
    here = os.path.dirname(os.path.abspath(__file__))
    csrc = os.path.join(os.path.dirname(here), "moeva2-ijcai22-replication_amd", "csrc")
    exe = str(tmp_path / "detpow_fma_check")
    subprocess.run([cxx, "-O2", "-ffp-contract=off", "-std=c++17", "-I", csrc,
                    os.path.join(here, "native", "detpow_fma_check.cpp"), "-o", exe],
                   check=True, capture_output=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout
