// node_visit_isa.hip -- the ISA of one BVH4 node visit, alone (tools/node_visit_isa.py counts it):
// a kernel around rt_hip.hip's node_visit<false, kF16> (the planes instance's visit, fp16 codes),
// compiled with the product flags to device assembly only.  Not part of the library.
#include "../ray_tracying_amd/csrc/hip/rt_hip.hip"

namespace {
__global__ __launch_bounds__(kBlock) void node_visit_probe(TraceArgs ta, const float* qin, int* out) {
  extern __shared__ __attribute__((aligned(16))) int lds_stack[];
  const int gtid = blockIdx.x * kBlock + threadIdx.x;
  Query q;
  setup_query(q, V3{qin[0], qin[1], qin[2]}, V3{qin[3 + gtid % 3], qin[4], qin[5]}, 0.0f, false);
  const LaneStack S{reinterpret_cast<char*>(lds_stack), reinterpret_cast<int2*>(ta.spill)};
  int w = (int)threadIdx.x * 8;
  unsigned nbox = 0, nvisit = 0;
  unsigned long long dg = 0;
  asm volatile("; NODE_VISIT_BEGIN" ::: "memory");
  const int item = node_visit<false, true>(ta, q, qin[6], out[gtid], S, w, gtid, nbox, dg, nvisit);
  asm volatile("; NODE_VISIT_END" ::: "memory");
  out[gtid] = item + w;
}
}  // namespace
void* node_visit_probe_ptr = (void*)&node_visit_probe;
