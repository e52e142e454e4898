"""CPU: the C-ABI library loads, exports every symbol include/sgx.h declares, and its
pure-host entry points (exchange planning, index helpers, errors) behave; no GPU calls."""
import os
import re
import struct

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from conftest import ROOT


def header_functions():
    txt = open(os.path.join(ROOT, "include", "sgx.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sgx_[a-z0-9_]+)\s*\(", txt)))


def test_every_declared_symbol_is_exported_and_bound(sgx_lib):
    names = header_functions()
    assert len(names) >= 30
    lib = sgx_lib.lib()
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/sgx.h but not exported"
        assert n in sgx_lib._lib.SIGNATURES, f"{n} has no ctypes signature"
    assert set(sgx_lib._lib.SIGNATURES) == set(names)
    assert lib.sgx_abi_version() == sgx_lib._lib.ABI_VERSION == 7


def test_library_is_gfx950_code_object():
    so = os.path.join(ROOT, "sparkucx_amd", "libsgx.so")
    data = open(so, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"k_scatter16" in data and b"k_scan" in data and b"k_hist" in data


def test_no_gpu_create_fails_loudly(sgx_lib):
    import torch

    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(sgx_lib.DeviceError):
        sgx_lib.ShuffleEngine(device=0)


def test_reducer_owner_contiguous(sgx_lib):
    for R in (1, 7, 200, 1024, 4096):
        for P in (1, 2, 3, 4, 8):
            own = [sgx_lib.reducer_owner(r, R, P) for r in range(R)]
            assert own == [(r * P) // R for r in range(R)]
            assert own == sorted(own)


def reference_plan(L, rank, item_bytes):
    """Independent restatement of the exchange plan for the test."""
    P, R = L.shape
    own = [(r * P) // R for r in range(R)]
    sc = np.zeros(P, np.int64)
    for r in range(R):
        sc[own[r]] += L[rank, r]
    mine = [r for r in range(R) if own[r] == rank]
    rc = np.array([sum(L[s, r] for r in mine) for s in range(P)], np.int64)
    rd = np.concatenate([[0], np.cumsum(rc)[:-1]]).astype(np.int64)
    items = []
    srun = rd.copy()
    dst = 0
    for r in mine:
        for s in range(P):
            ln = int(L[s, r])
            so = int(srun[s])
            srun[s] += ln
            while ln > 0:
                piece = min(ln, item_bytes) if item_bytes else ln
                items.append((so, dst, piece))
                so += piece
                dst += piece
                ln -= piece
    return sc, np.concatenate([[0], np.cumsum(sc)[:-1]]), rc, rd, np.array(items, np.int64).reshape(-1, 3)


@settings(max_examples=60, deadline=None)
@given(P=st.integers(1, 8), R=st.integers(1, 64), item=st.sampled_from([0, 16, 48, 4096]),
       seed=st.integers(0, 2**31 - 1))
def test_plan_exchange_matches_restatement(sgx_lib, P, R, item, seed):
    rng = np.random.default_rng(seed)
    L = (rng.integers(0, 5, size=(P, R)) * 16).astype(np.int64)
    for rank in range(P):
        got = sgx_lib.plan_exchange(L, rank, item)
        want = reference_plan(L, rank, item)
        for g, w in zip(got, want):
            assert np.array_equal(np.asarray(g).reshape(np.asarray(w).shape), w)
    # conservation: what rank j sends to k is what k receives from j
    plans = [sgx_lib.plan_exchange(L, r, 0) for r in range(P)]
    for j in range(P):
        for k in range(P):
            assert plans[j][0][k] == plans[k][2][j]


def test_plan_exchange_rejects_bad_args(sgx_lib):
    with pytest.raises(sgx_lib.IllegalArgumentException):
        sgx_lib.plan_exchange(np.zeros((2, 4), np.int64), 5)


def write_files(tmp_path, lengths, data_len=None):
    import oracle

    idx = tmp_path / "shuffle_0_0_0.index"
    dat = tmp_path / "shuffle_0_0_0.data"
    idx.write_bytes(oracle.index_bytes(np.asarray(lengths, np.int64)))
    dat.write_bytes(b"\0" * (sum(lengths) if data_len is None else data_len))
    return str(idx), str(dat)


def test_check_index_and_data_host_helper(sgx_lib, tmp_path):
    lib = sgx_lib.lib()
    lengths = [16, 0, 48, 32]
    idx, dat = write_files(tmp_path, lengths)
    out = np.zeros(4, np.int64)
    assert lib.sgx_check_index_and_data(idx.encode(), dat.encode(), 4, out.ctypes.data) == 0
    assert out.tolist() == lengths
    assert lib.sgx_check_index_and_data(idx.encode(), dat.encode(), 3, out.ctypes.data) == sgx_lib._lib.SGX_ERR_NOT_FOUND
    idx2, dat2 = write_files(tmp_path, lengths, data_len=95)
    assert lib.sgx_check_index_and_data(idx2.encode(), dat2.encode(), 4, out.ctypes.data) != 0


def test_index_block_range_host_helper(sgx_lib, tmp_path):
    import ctypes

    lib = sgx_lib.lib()
    idx, _ = write_files(tmp_path, [16, 0, 48, 32])
    off, ln = ctypes.c_int64(), ctypes.c_int64()
    assert lib.sgx_index_block_range(idx.encode(), 2, 3, ctypes.byref(off), ctypes.byref(ln)) == 0
    assert (off.value, ln.value) == (16, 48)
    assert lib.sgx_index_block_range(idx.encode(), 0, 4, ctypes.byref(off), ctypes.byref(ln)) == 0
    assert (off.value, ln.value) == (0, 96)
    assert lib.sgx_index_block_range(idx.encode(), 3, 9, ctypes.byref(off), ctypes.byref(ln)) == sgx_lib._lib.SGX_ERR_IO


def test_block_id_wire_format(sgx_lib):
    b = sgx_lib.UcxShuffleBlockId(3, 5, 1023)
    assert b.serialize() == struct.pack(">ii", 5, 1023)
    assert sgx_lib.UcxShuffleBlockId.deserialize(b.serialize()) == sgx_lib.UcxShuffleBlockId(0, 5, 1023)
    assert sgx_lib.parse_block_id("shuffle_1_22_333") == (1, 22, 333)
    with pytest.raises(sgx_lib.IllegalArgumentException):
        sgx_lib.parse_block_id("rdd_1_2")


def test_partitioner_types(sgx_lib):
    assert sgx_lib.HashPartitioner(200).numPartitions == 200
    with pytest.raises(sgx_lib.IllegalArgumentException):
        sgx_lib.HashPartitioner(-1)
    rp = sgx_lib.RangePartitioner(np.array([1, 5, 9], np.int64))
    assert rp.numPartitions == 4 and rp.kind == sgx_lib.PART_RANGE_I64
    rb = sgx_lib.RangePartitioner(np.zeros((7, 10), np.uint8))
    assert rb.numPartitions == 8 and rb.kind == sgx_lib.PART_RANGE_BYTES10


def test_map_output_writer_contract(sgx_lib):
    w = sgx_lib.GpuShuffleMapOutputWriter(0, 1, np.array([16, 0, 32], np.int64))
    assert w.getPartitionWriter(0).getNumBytesWritten() == 16
    assert w.getPartitionWriter(2).getNumBytesWritten() == 32
    with pytest.raises(sgx_lib.IllegalArgumentException, match="increasing order"):
        w.getPartitionWriter(1)
    assert w.commitAllPartitions().tolist() == [16, 0, 32]


def test_check_index_accepts_decreasing_offsets_like_spark(sgx_lib, oracle_lib, tmp_path):
    """IndexShuffleBlockResolver.checkIndexAndDataFile (:110-149) checks the long count, the
    first offset and that the lengths sum to the data size -- nothing else.  An index with a
    decreasing offset (a negative length) whose lengths still sum to the data file's size is
    valid, for the engine as for the restatement (oracle/spark_semantics.py)."""
    import struct

    from oracle import spark_semantics as S

    offs = [0, 64, 16, 80, 96]  # lengths 64, -48, 64, 16: sum 96
    idxb = b"".join(struct.pack(">q", o) for o in offs)
    idx, dat = tmp_path / "d.index", tmp_path / "d.data"
    idx.write_bytes(idxb)
    dat.write_bytes(b"\1" * 96)
    out = np.zeros(4, np.int64)
    assert sgx_lib.lib().sgx_check_index_and_data(str(idx).encode(), str(dat).encode(), 4, out.ctypes.data) == 0
    assert out.tolist() == [64, -48, 64, 16] == S.check_index_and_data(idxb, 96, 4)
    dat.write_bytes(b"\1" * 80)
    assert sgx_lib.lib().sgx_check_index_and_data(str(idx).encode(), str(dat).encode(), 4, out.ctypes.data) != 0
    assert S.check_index_and_data(idxb, 80, 4) is None


def test_header_enum_and_flag_values_match_the_bindings(sgx_lib):
    """Every `SGX_<NAME> = value` of include/sgx.h's enums that the Python bindings also
    define (as <NAME>) carries the same value, e.g. the map layouts and engine flags."""
    import sparkucx_amd._lib as L

    txt = open(os.path.join(ROOT, "include", "sgx.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    pairs = re.findall(r"\bSGX_([A-Z0-9_]+)\s*=\s*(-?\d+)\b", txt)
    assert pairs, "no enum values parsed from include/sgx.h"
    checked = 0
    for name, val in pairs:
        if hasattr(L, name):
            assert getattr(L, name) == int(val), f"SGX_{name} = {val} in sgx.h, {getattr(L, name)} in _lib"
            checked += 1
    assert checked >= 10
    assert L.LAYOUT_SERIALIZED_PADDED == 2
