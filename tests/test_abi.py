"""The C-ABI library loads without a GPU and exports every function include/ocppo.h declares;
argument validation and the error channel work without launching anything."""
import ctypes
import re

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def lib():
    from oc_cleanrl_amd import _lib

    return _lib


def test_header_functions_exported(lib):
    names = lib.header_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib.LIB, n), f"{n} declared in include/ocppo.h but not exported"
        assert n in lib.SIGNATURES, f"{n} has no ctypes signature"
    assert set(lib.SIGNATURES) == set(names)


def test_header_constants_match_python(lib):
    text = (ROOT / "include" / "ocppo.h").read_text()
    consts = dict(re.findall(r"#define (OCPPO_\w+) (\d+)", text))
    assert int(consts["OCPPO_ABI_VERSION"]) == lib.OCPPO_ABI_VERSION == lib.LIB.ocppo_abi_version()
    assert int(consts["OCPPO_F32"]) == lib.OCPPO_F32
    assert int(consts["OCPPO_BF16"]) == lib.OCPPO_BF16
    assert int(consts["OCPPO_U8"]) == lib.OCPPO_U8
    assert int(consts["OCPPO_NUM_STATS"]) == lib.OCPPO_NUM_STATS
    stat_names = re.findall(r"#define OCPPO_STAT_(\w+) (\d+)", text)
    assert [n.lower() for n, _ in sorted(stat_names, key=lambda x: int(x[1]))] == list(lib.STAT_NAMES)


def test_only_c_abi_is_exported():
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only",
                          str(ROOT / "oc_cleanrl_amd" / "lib" / "libocppo_hip.so")],
                         capture_output=True, text=True, check=True).stdout
    syms = [l.split()[-1] for l in out.splitlines() if l.split()[1] in ("T", "D", "B", "W", "V")]
    assert all(s.startswith("ocppo_") for s in syms), [s for s in syms if not s.startswith("ocppo_")]


def test_invalid_arguments_report_errors_without_launch(lib):
    L = lib.LIB
    rc = L.ocppo_gae(None, None, None, None, None, None, 8, 4, 0.99, 0.95, None, None)
    assert rc == lib.OCPPO_E_INVALID
    assert b"null pointer" in L.ocppo_last_error()
    rc = L.ocppo_ppo_loss_fwd_bwd(None, None, None, 16, 64, *([None] * 7), 0.1, 0.01, 0.5, 1, 1,
                                  None, None, None, None, 0)
    assert rc == lib.OCPPO_E_INVALID and b"A <= 32" in L.ocppo_last_error()
    dummy = ctypes.c_void_p(16)
    rc = L.ocppo_ppo_loss_fwd_bwd(None, dummy, dummy, 16, 6, None, dummy, dummy, dummy, dummy,
                                  dummy, None, 0.1, 0.01, 0.5, 1, 1, dummy, dummy, dummy, None, 0)
    assert rc == lib.OCPPO_E_WORKSPACE
    with pytest.raises(lib.OcppoError, match="ocppo_gather_rows"):
        lib.call("ocppo_gather_rows", None, None, 7, None, 4, 4, None)


def test_deferred_finish_record_is_checked(lib):
    """ocppo_deferred_finish_run / ocppo_sum_splits_finish refuse a missing record or one no
    ocppo_heads_loss_rows call filled, before any launch."""
    L = lib.LIB
    assert L.ocppo_deferred_finish_run(None, None) == lib.OCPPO_E_INVALID
    assert b"null finish record" in L.ocppo_last_error()
    rec = (ctypes.c_uint64 * 64)()
    assert L.ocppo_deferred_finish_run(None, ctypes.addressof(rec)) == lib.OCPPO_E_INVALID
    assert b"not a finish record" in L.ocppo_last_error()
    dummy = ctypes.c_void_p(256)
    assert L.ocppo_sum_splits_finish(None, dummy, 8, 1024, dummy,
                                     ctypes.addressof(rec)) == lib.OCPPO_E_INVALID
    assert b"not a finish record" in L.ocppo_last_error()
    assert L.ocppo_sum_splits_finish(None, dummy, 3, 1024, dummy,
                                     ctypes.addressof(rec)) == lib.OCPPO_E_INVALID
    assert b"bad sizes" in L.ocppo_last_error()


def test_zero_sized_calls_are_noops(lib):
    assert lib.LIB.ocppo_gae(None, None, None, None, None, None, 0, 0, 0.99, 0.95, None, None) == 0
    assert lib.LIB.ocppo_gather_rows(None, None, 0, None, 0, 4, None) == 0


def test_workspace_size_is_host_only(lib):
    n = lib.LIB.ocppo_ppo_loss_workspace_bytes(4096, 6)
    assert n >= 256 + 16 * 6 * 4 and n % 16 == 0


def test_library_reads_no_environment():
    """No tiling, grid or workspace choice of the shipped library depends on the environment:
    it imports no getenv (the geometry knobs of experiments are compile-time -D flags for
    tools/build_variant.py, or explicit ABI arguments such as ocppo_gemm_x6's mbig)."""
    import subprocess

    out = subprocess.run(["nm", "-D", "--undefined-only",
                          str(ROOT / "oc_cleanrl_amd" / "lib" / "libocppo_hip.so")],
                         capture_output=True, text=True, check=True).stdout
    assert not [l for l in out.splitlines() if "getenv" in l]
    for src in (ROOT / "oc_cleanrl_amd" / "csrc").glob("*.hip"):
        assert "getenv" not in src.read_text(), src.name


def test_gemm_x6_mbig_only_for_the_mixed_tile(lib):
    dummy = ctypes.c_void_p(256)
    args = [None, dummy, 64, 1, dummy, 64, 1, dummy, 128, 128, 128, 64, 1, 0, None, 0, None, 0,
            None, None, None]
    assert lib.LIB.ocppo_gemm_x6(*args, 24, 512, None, 0, 0, None, 0) == lib.OCPPO_E_INVALID
    assert b"mbig" in lib.LIB.ocppo_last_error()


def test_gemm_x6_rejects_operand_windows_past_32_bit_offsets(lib):
    """The x6 kernels address a tile's operand window with 32-bit buffer offsets: a row stride
    that puts one 128-row window past 2 GiB is refused before any launch (validation only)."""
    dummy = ctypes.c_void_p(256)
    ok = [None, dummy, 64, 1, dummy, 64, 1, dummy, 128, 128, 128, 64, 1, 0, None, 0, None, 0,
          None, None, None, 24, -1, None, 0, 0, None, 0]
    big = list(ok)
    big[2] = 1 << 22  # A row stride 4M floats: 256 rows x 16 MB
    assert lib.LIB.ocppo_gemm_x6(*big) == lib.OCPPO_E_INVALID
    assert b"2 GiB" in lib.LIB.ocppo_last_error()
