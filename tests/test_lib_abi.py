"""CPU-only checks of the C ABI: libfedcodec.so loads, exports every symbol include/fedcodec.h
declares, struct layouts agree, and argument errors surface without touching a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fedcodec.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fc_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from openmsftl_amd import build, _lib
    build.build(verbose=False)
    return _lib.load()


def test_header_declares_expected_surface():
    names = _declared()
    for must in ("fc_topk_encode", "fc_topk_encode_exact", "fc_mask_encode", "fc_decode_dense",
                 "fc_decode_accumulate", "fc_weighted_sum_dense", "fc_workspace_bytes"):
        assert must in names


def test_every_declared_symbol_is_exported(lib):
    from openmsftl_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\s[TW]\s+(\S+)", out))
    for name in _declared():
        assert name in exported, name
        assert name in _lib.SIGNATURES, f"{name} not bound in _lib.SIGNATURES"
        getattr(lib, name)


def test_lib_is_gfx950_only():
    from openmsftl_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    triples = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert triples == {b"gfx950"}, triples


def test_struct_layouts():
    from openmsftl_amd import _lib
    assert ctypes.sizeof(_lib.PacketHdr) == 96
    assert ctypes.sizeof(_lib.PacketView) == 56
    assert _lib.PacketHdr.p.offset == 64 and _lib.PacketHdr.seed.offset == 48
    assert _lib.PacketView.cnt.offset == 24 and _lib.PacketView.qoff.offset == 40
    assert _lib.PacketView.weight.offset == 48
    assert ctypes.sizeof(_lib.EncodeJob) == 64 and _lib.EncodeJob.qoff.offset == 56


def test_sizes_are_host_functions(lib):
    assert lib.fc_num_chunks(1) == 1 and lib.fc_num_chunks(8192) == 1
    assert lib.fc_num_chunks(8193) == 2
    assert lib.fc_workspace_bytes(1 << 27) > 8 * lib.fc_num_chunks(1 << 27)
    assert lib.fc_packet_capacity(134_217_728) == 134_217_728
    assert lib.fc_packet_capacity(1000) == 8192


def test_argument_errors_do_not_touch_gpu(lib):
    from openmsftl_amd import _lib
    rc = lib.fc_topk_encode(None, 10, 1, 0, 0, 0, None, None, 10, None, None, None, None, 0, None)
    assert rc == -1 and b"g is NULL" in lib.fc_last_error()
    buf = ctypes.create_string_buffer(64)
    addr = (ctypes.addressof(buf) + 15) & ~15
    rc = lib.fc_topk_encode(addr, 10, 1, 0, 0, 0, addr, addr, 10, addr, addr, addr, addr, 16, None)
    assert rc == -3 and b"workspace" in lib.fc_last_error()
    rc = lib.fc_mask_encode(addr, 10, 99, None, 0.5, 0, 0, 1, None, addr, addr, 10, addr, None,
                            addr, addr, 1 << 20, None)
    assert rc == -1 and b"bad codec" in lib.fc_last_error()
    with pytest.raises(_lib.FedCodecError):
        _lib.check(lib.fc_decode_accumulate(None, 1, 0, 10, None, None), "decode_accumulate")


def test_flat_stage_argument_errors(lib):
    buf = ctypes.create_string_buffer(64)
    addr = (ctypes.addressof(buf) + 15) & ~15
    assert lib.fc_flat_stage(None, addr, 1, 1, addr, None, 0, None) == -1
    assert lib.fc_flat_stage(addr, addr, 0, 1, addr, None, 0, None) == -1
    assert b"count" in lib.fc_last_error()
    assert lib.fc_flat_stage(addr, addr, 1, 1, addr, addr, 1, None) == -1
    assert b"scatter" in lib.fc_last_error()
