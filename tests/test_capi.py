"""CPU-side checks of the C-ABI library (no GPU compute): it loads, exports every symbol include/pfmpe.h
declares, and its host-evaluated RNG code (the same __host__ __device__ functions the kernels run)
matches the oracle's libstdc++ stream and the Philox KATs."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import _capi
from oracle import pforacle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    hdr = open(os.path.join(ROOT, "include", "pfmpe.h")).read()
    return sorted(set(re.findall(r"\b(pfmpe_[a-z_0-9]+)\s*\(", hdr)))


def test_header_declarations_match_binding():
    assert sorted(_capi.EXPORTED_SYMBOLS) == declared_functions()


def test_library_exports_every_declared_symbol():
    lib = pf.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", pf.LIB_PATH], capture_output=True, text=True, check=True).stdout
    for name in declared_functions():
        assert re.search(rf"\bT {name}\b", nm), name


def test_abi_version_and_defaults():
    lib = pf.load()
    assert lib.pfmpe_abi_version() == 1
    p = pf.default_params()
    assert (p.tol, p.tol_pf, p.max_iter, p.exit_cap, p.accept_cap) == (5.0, 4.0, 80, 5, 3)
    assert p.growth == 0.025 and p.ang_max == 0.015 and p.trans_max == 0.035


def test_struct_layouts():
    assert ctypes.sizeof(_capi.FrameOut) == 4 * 8 + 8 * 2 + 8 * 24 + 4 * 32
    assert ctypes.sizeof(_capi.Params) == 7 * 8 + 4 * 4


@pytest.mark.parametrize("seed", [0, 1, 42, 2**31 - 2, 2**31 - 1, 2**32 - 1])
def test_host_jump_ahead_equals_libstdcxx_stream(seed):
    a, b = -0.0035, 0.0035
    ref = orc.uniform_draws(seed, a, b, 300)
    got = np.array([pf.host_ref_uniform(seed, j, a, b) for j in range(300)])
    assert np.array_equal(ref, got)


def test_host_jump_far_ahead():
    # draw 2^20 + 5 via the oracle's sequential stream vs direct jump
    n = (1 << 16) + 5
    ref = orc.uniform_draws(99, 0.0, 1.0, n)
    assert pf.host_ref_uniform(99, n - 1, 0.0, 1.0) == ref[-1]


def test_host_philox_matches_oracle_and_kat():
    assert pf.host_philox([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    rng = np.random.default_rng(1)
    for _ in range(50):
        c = [int(x) for x in rng.integers(0, 2**32, 4)]
        k = [int(x) for x in rng.integers(0, 2**32, 2)]
        assert pf.host_philox(c, k) == orc.philox(c, k)


def test_create_without_gpu_fails_cleanly():
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU driver is present")
    with pytest.raises(pf.PFError):
        pf.Engine(device=0, max_particles=10)
