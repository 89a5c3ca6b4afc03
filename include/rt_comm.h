/* rt_comm.h -- C ABI of librt_comm.so: RCCL (over xGMI) collectives for the multi-GPU
 * image-tile path ("rt_gather_rccl").
 *
 * The reference renders one image on one core (raytracer.cpp:433-476) and has no
 * communication at all; this layer exists for the replacement's tile parallelism: every
 * device renders its tiles (rt_render_tiles) into a packed device buffer, and one grouped
 * ncclGather collects the buffers on the root device.  Single process, one communicator
 * rank per listed device (ncclCommInitAll).  Multi-process runs (bench.py) use
 * torch.distributed over the same RCCL instead.
 *
 * Conventions as rt_hip.h: 0 = success, negative RT_E* codes, rt_comm_last_error() is
 * thread-local, no exceptions cross the ABI. */
#ifndef RT_COMM_H
#define RT_COMM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_comm_s* rt_comm_t;

/* One rank per entry of devices[0..n_devices-1] (distinct HIP device ids). */
int rt_comm_create(int32_t n_devices, const int32_t* devices, rt_comm_t* out);
int rt_comm_destroy(rt_comm_t comm);
int rt_comm_size(rt_comm_t comm, int32_t* n);

/* Gather count floats from d_send[r] (a buffer on device devices[r]) of every rank r into
 * d_recv (on devices[root], n_devices * count floats, rank-major).  Blocks until done. */
int rt_comm_gather_f32(rt_comm_t comm, const float* const* d_send, size_t count, float* d_recv, int32_t root);

const char* rt_comm_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
