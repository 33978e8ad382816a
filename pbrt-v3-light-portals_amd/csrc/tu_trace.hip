// tu_trace.hip -- translation unit of the BVH traversal kernels (kernels.hip).
#define PT_TU_TRACE 1
#include "kernels.hip"

namespace pt {
#define PT_ARGS DevScene, DevPaths, const uint32_t*, const uint32_t*
template __global__ void k_trace<false, false>(PT_ARGS, int*, DevStats*);
template __global__ void k_trace<false, true>(PT_ARGS, int*, DevStats*);
template __global__ void k_trace<true, false>(PT_ARGS, int*, DevStats*);
template __global__ void k_trace<true, true>(PT_ARGS, int*, DevStats*);
template __global__ void k_trace_nb<false, false>(PT_ARGS, uint32_t*, int, int, DevStats*);
template __global__ void k_trace_nb<false, true>(PT_ARGS, uint32_t*, int, int, DevStats*);
template __global__ void k_trace_nb<true, false>(PT_ARGS, uint32_t*, int, int, DevStats*);
template __global__ void k_trace_nb<true, true>(PT_ARGS, uint32_t*, int, int, DevStats*);
template __global__ void k_trace_lds<false>(PT_ARGS, uint32_t*, int, int, DevStats*);
template __global__ void k_trace_lds<true>(PT_ARGS, uint32_t*, int, int, DevStats*);
template __global__ void k_trace_oct<false>(PT_ARGS, uint32_t*, int, int, DevStats*);
template __global__ void k_trace_oct<true>(PT_ARGS, uint32_t*, int, int, DevStats*);
template __global__ void k_trace_w<false>(PT_ARGS, uint32_t*, int, int, uint32_t*, uint32_t*, int, uint32_t*, DevStats*);
template __global__ void k_trace_w<true>(PT_ARGS, uint32_t*, int, int, uint32_t*, uint32_t*, int, uint32_t*, DevStats*);
#define PT_PT(a, b, c) template __global__ void k_trace_pt<a, b, c>(PT_ARGS, uint32_t*, int, int, int, int*, DevStats*);
PT_PT(false, false, false) PT_PT(false, false, true) PT_PT(false, true, false) PT_PT(false, true, true)
PT_PT(true, false, false) PT_PT(true, false, true) PT_PT(true, true, false) PT_PT(true, true, true)
#undef PT_PT
#undef PT_ARGS
}  // namespace pt
