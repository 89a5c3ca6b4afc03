// rt_comm.cpp -- RCCL collectives for the image-tile path (include/rt_comm.h).
#include "../../../include/rt_comm.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>
#include <vector>

#include "../../../include/rt_hip.h"

namespace {
thread_local std::string g_err;
int fail(int code, const std::string& m) {
  g_err = m;
  return code;
}
}  // namespace

struct rt_comm_s {
  std::vector<int> devices;
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> streams;
};

extern "C" {

const char* rt_comm_last_error(void) { return g_err.c_str(); }

int rt_comm_create(int32_t n, const int32_t* devices, rt_comm_t* out) {
  if (n < 1 || !devices || !out) return fail(RT_EINVAL, "rt_comm_create: bad argument");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) return fail(RT_ENODEV, "rt_comm_create: no HIP device");
  for (int i = 0; i < n; ++i) {
    if (devices[i] < 0 || devices[i] >= ndev) return fail(RT_ENODEV, "rt_comm_create: no such device");
    for (int j = 0; j < i; ++j)
      if (devices[j] == devices[i]) return fail(RT_EINVAL, "rt_comm_create: devices must be distinct");
  }
  auto* c = new rt_comm_s();
  c->devices.assign(devices, devices + n);
  c->comms.resize(n);
  ncclResult_t r = ncclCommInitAll(c->comms.data(), n, c->devices.data());
  if (r != ncclSuccess) {
    delete c;
    return fail(RT_EDEVICE, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
  }
  c->streams.resize(n);
  for (int i = 0; i < n; ++i) {
    if (hipSetDevice(c->devices[i]) != hipSuccess || hipStreamCreate(&c->streams[i]) != hipSuccess) {
      rt_comm_destroy(c);
      return fail(RT_EDEVICE, "rt_comm_create: stream");
    }
  }
  *out = c;
  return RT_OK;
}

int rt_comm_destroy(rt_comm_t c) {
  if (!c) return RT_OK;
  for (size_t i = 0; i < c->comms.size(); ++i)
    if (c->comms[i]) ncclCommDestroy(c->comms[i]);
  for (size_t i = 0; i < c->streams.size(); ++i)
    if (c->streams[i]) {
      (void)hipSetDevice(c->devices[i]);
      (void)hipStreamDestroy(c->streams[i]);
    }
  delete c;
  return RT_OK;
}

int rt_comm_size(rt_comm_t c, int32_t* n) {
  if (!c || !n) return fail(RT_EINVAL, "rt_comm_size: null argument");
  *n = (int32_t)c->devices.size();
  return RT_OK;
}

int rt_comm_gather_f32(rt_comm_t c, const float* const* d_send, size_t count, float* d_recv, int32_t root) {
  if (!c || !d_send || root < 0 || root >= (int)c->devices.size() || (!d_recv && count))
    return fail(RT_EINVAL, "rt_comm_gather_f32: bad argument");
  const int n = (int)c->devices.size();
  ncclResult_t r = ncclGroupStart();
  for (int i = 0; i < n && r == ncclSuccess; ++i) {
    (void)hipSetDevice(c->devices[i]);
    r = ncclGather(d_send[i], i == root ? d_recv : nullptr, count, ncclFloat32, root, c->comms[i], c->streams[i]);
  }
  ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess || r2 != ncclSuccess)
    return fail(RT_EDEVICE, std::string("ncclGather: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
  for (int i = 0; i < n; ++i) {
    (void)hipSetDevice(c->devices[i]);
    if (hipStreamSynchronize(c->streams[i]) != hipSuccess) return fail(RT_EDEVICE, "rt_comm_gather_f32: sync");
  }
  return RT_OK;
}

}  // extern "C"
