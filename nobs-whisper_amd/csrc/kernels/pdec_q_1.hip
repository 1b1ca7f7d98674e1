// Persistent decode step, half_t GGML-block weights, built for 1 row (one translation unit per
// instantiation set: they build in parallel)
#include "pdec_body.h"

namespace wm {
void pdec_launch_q_1(const PdecArgs& a, size_t lds, hipStream_t st) { pdec_launch_t<half_t, true, 1>(a, lds, st); }
}  // namespace wm
