// Persistent decode step, half_t GGML-block weights, built for 4 rows (one translation unit per
// instantiation set: they build in parallel)
#include "pdec_body.h"

namespace wm {
void pdec_launch_q_4(const PdecArgs& a, size_t lds, hipStream_t st) { pdec_launch_t<half_t, true, 4>(a, lds, st); }
}  // namespace wm
