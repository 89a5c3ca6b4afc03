"""librt_comm.so (include/rt_comm.h): the RCCL gather of packed tile buffers used by the
C++ CLI's -gpus N path.  On a one-GPU box the communicator has one rank,
so the gather is a device-to-device copy through RCCL; argument checking runs on CPU."""
import ctypes
import os

import numpy as np
import pytest

import ray_tracying_amd as rt

LIB = os.path.join(rt.LIB_DIR, "librt_comm.so")


def comm_lib():
    L = ctypes.CDLL(LIB)
    L.rt_comm_last_error.restype = ctypes.c_char_p
    return L


def test_comm_rejects_bad_arguments():
    L = comm_lib()
    out = ctypes.c_void_p()
    assert L.rt_comm_create(0, None, ctypes.byref(out)) < 0
    devs = (ctypes.c_int32 * 2)(0, 0)
    # duplicate devices are refused before any device is touched (or: no device here)
    assert L.rt_comm_create(2, devs, ctypes.byref(out)) < 0
    assert L.rt_comm_last_error()


@pytest.mark.gpu
def test_gather_one_rank_roundtrip(gpu):
    L = comm_lib()
    H = rt.hip_lib()
    n = 3 * 64 * 64 * 5
    src = (np.arange(n, dtype=np.float32) * 0.5 - 7.0)
    d_src, d_dst = ctypes.c_void_p(), ctypes.c_void_p()
    assert H.rt_malloc(0, n * 4, ctypes.byref(d_src)) == 0
    assert H.rt_malloc(0, n * 4, ctypes.byref(d_dst)) == 0
    try:
        assert H.rt_memcpy_h2d(d_src, src.ctypes.data_as(ctypes.c_void_p), n * 4) == 0
        comm = ctypes.c_void_p()
        devs = (ctypes.c_int32 * 1)(0)
        assert L.rt_comm_create(1, devs, ctypes.byref(comm)) == 0, L.rt_comm_last_error()
        size = ctypes.c_int32()
        assert L.rt_comm_size(comm, ctypes.byref(size)) == 0 and size.value == 1
        sends = (ctypes.c_void_p * 1)(d_src.value)
        assert L.rt_comm_gather_f32(comm, sends, ctypes.c_size_t(n), d_dst, 0) == 0, L.rt_comm_last_error()
        out = np.empty(n, dtype=np.float32)
        assert H.rt_memcpy_d2h(out.ctypes.data_as(ctypes.c_void_p), d_dst, n * 4) == 0
        assert np.array_equal(out.view(np.uint32), src.view(np.uint32))
        assert L.rt_comm_destroy(comm) == 0
    finally:
        H.rt_free(d_src)
        H.rt_free(d_dst)
