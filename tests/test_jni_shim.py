"""CPU: the JNI shim (jni/sgx_jni.c) compiled against jni/stub/jni.h and linked with
libsgx.so, driven through a fake JNIEnv (tests/native/jni_fake_env.c) via ctypes.  Covers
the natives that need no GPU and the error -> exception mapping the Scala side relies on
(SURVEY §8(b) error conventions; FetchFailed for failed fetches, which the reference never
raises, spark_3_0/UcxShuffleClient.scala:36-40)."""
import ctypes
import os
import shutil
import socket
import subprocess
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def shim(sgx_lib, tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("needs gcc")
    out = str(tmp_path_factory.mktemp("jni") / "libjnitest.so")
    lib_dir = os.path.join(ROOT, "sparkucx_amd")
    subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-shared", "-fPIC",
                    "-I" + os.path.join(ROOT, "jni", "stub"), "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "jni", "sgx_jni.c"), os.path.join(ROOT, "tests", "native", "jni_fake_env.c"),
                    "-L" + lib_dir, "-l:libsgx.so", "-Wl,-rpath," + lib_dir, "-o", out], check=True)
    L = ctypes.CDLL(out)
    L.fake_exception_class.restype = ctypes.c_char_p
    L.fake_exception_message.restype = ctypes.c_char_p
    L.fake_check_index.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p]
    L.fake_index_block_range.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.fake_write_map.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
    L.fake_fetch_mismatched.argtypes = [ctypes.c_int64]
    L.fake_exchange.argtypes = [ctypes.c_int64]
    L.fake_import_blocks.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    L.fake_import_blocks.restype = ctypes.c_int64
    L.fake_exchange_fail.argtypes = [ctypes.c_int64, ctypes.c_int]
    L.fake_exchange_maps.argtypes = [ctypes.c_int64, ctypes.c_int]
    L.fake_set_map_writer.argtypes = [ctypes.c_int64, ctypes.c_int]
    L.fake_shuffle_reducers.argtypes = [ctypes.c_int64, ctypes.c_void_p]
    L.fake_bootstrap_join.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p]
    L.fake_bootstrap_serve.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    return L


def exc(shim):
    return shim.fake_exception_class().decode(), shim.fake_exception_message().decode()


def test_index_natives(shim, oracle_lib, tmp_path):
    lengths = np.array([0, 32, 16, 0, 48], np.int64)
    idx, dat = tmp_path / "shuffle_1_0_0.index", tmp_path / "shuffle_1_0_0.data"
    idx.write_bytes(oracle_lib.index_bytes(lengths))
    dat.write_bytes(bytes(96))
    out = np.zeros(5, np.int64)
    shim.fake_clear()
    assert shim.fake_check_index(str(idx).encode(), str(dat).encode(), 5, out.ctypes.data) == 5
    assert np.array_equal(out, lengths) and exc(shim) == ("", "")
    # a mismatch is Java null, not an exception (checkIndexAndDataFile returns null)
    assert shim.fake_check_index(str(idx).encode(), str(dat).encode(), 4, out.ctypes.data) == -1
    assert exc(shim)[0] == ""
    r = np.zeros(2, np.int64)
    assert shim.fake_index_block_range(str(idx).encode(), 1, 3, r.ctypes.data) == 0
    assert list(r) == [0, 48]
    assert shim.fake_index_block_range(str(tmp_path / "missing.index").encode(), 0, 1, r.ctypes.data) == -1
    assert exc(shim)[0] == "java/io/IOException"


def test_argument_errors_become_illegal_argument(shim):
    rec = np.zeros(64, np.uint8)
    shim.fake_clear()
    assert shim.fake_write_map(0, rec.ctypes.data, rec.nbytes, 4, 0) == -1  # numPartitions 0
    assert exc(shim)[0] == "java/lang/IllegalArgumentException"
    shim.fake_clear()
    assert shim.fake_write_map(0, rec.ctypes.data, rec.nbytes, 100, 8) == -1  # buffer too small
    assert exc(shim)[0] == "java/lang/IllegalArgumentException"
    shim.fake_clear()
    assert shim.fake_write_map(0, rec.ctypes.data, rec.nbytes, 4, 8) == -1  # NULL engine -> SGX_ERR_INVALID
    assert exc(shim) == ("java/lang/IllegalArgumentException", "engine is NULL")
    shim.fake_clear()
    assert shim.fake_fetch_mismatched(0) == -1
    assert exc(shim)[0] == "java/lang/IllegalArgumentException"
    shim.fake_clear()
    shim.fake_exchange(0)
    assert exc(shim)[0] == "java/lang/IllegalArgumentException"
    # the per-shuffle exchange's natives (GpuExchangeCoordinator, GpuShuffleReader)
    for n in (0, 3):
        shim.fake_clear()
        shim.fake_exchange_maps(0, n)
        assert exc(shim)[0] == "java/lang/IllegalArgumentException", n
    shim.fake_clear()
    r = np.zeros(2, np.int32)
    assert shim.fake_shuffle_reducers(0, r.ctypes.data) == -1
    assert exc(shim)[0] == "java/lang/IllegalArgumentException"
    # blocks fetched from the owners (GpuShuffleReader.readRemote): one length per (reducer,
    # map) block, lengths within the buffer, then the engine's own checks
    buf = np.zeros(64, np.uint8)
    for r1, nlen, cap in ((2, 3, 64), (2, 4, 32), (2, 4, 64)):
        shim.fake_clear()
        assert shim.fake_import_blocks(0, buf.ctypes.data, cap, r1, nlen) == -1
        cls, m = exc(shim)
        assert cls == "java/lang/IllegalArgumentException", (r1, nlen, cap)
        if (nlen, cap) == (3, 64):
            assert "one length per" in m
        elif cap == 32:
            assert "exceed" in m
        else:
            assert "bad arguments" in m  # NULL engine, reported by sgx_import_blocks
    shim.fake_clear()
    shim.fake_exchange_fail(0, 8)
    assert exc(shim)[0] == "java/lang/IllegalArgumentException"
    # the handle's map writer (GpuUcxShuffleManager: UnsafeShuffleWriter for a SerializedShuffleHandle)
    for w in (0, 1):
        shim.fake_clear()
        shim.fake_set_map_writer(0, w)
        assert exc(shim)[0] == "java/lang/IllegalArgumentException", w


def test_bootstrap_natives_and_fetch_failure_mapping(shim):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    idb = (ctypes.c_uint8 * 128)(*range(128))
    got = (ctypes.c_uint8 * 128)()
    nr = ctypes.c_int(0)
    t = threading.Thread(target=shim.fake_bootstrap_serve, args=(port, 2, idb, 10_000))
    t.start()
    shim.fake_clear()
    assert shim.fake_bootstrap_join(b"127.0.0.1", port, 1, 10_000, got, ctypes.byref(nr)) == 0
    t.join()
    assert bytes(got) == bytes(idb) and nr.value == 2 and exc(shim)[0] == ""
    # nobody serving: the timeout is a fetch failure on the Scala side (stage retry)
    shim.fake_clear()
    assert shim.fake_bootstrap_join(b"127.0.0.1", port, 1, 300, got, ctypes.byref(nr)) == -1
    assert exc(shim)[0] == "org/apache/spark/shuffle/ucx/gpu/SgxFetchException"
