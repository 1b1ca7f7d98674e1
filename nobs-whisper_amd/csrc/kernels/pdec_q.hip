// Persistent decode step, half_t GGML-block weights (one translation unit per instantiation set: they build in parallel)
#include "pdec_body.h"

namespace wm {
void pdec_launch_q(const PdecArgs& a, size_t lds, hipStream_t st) { pdec_launch_t<half_t, true>(a, lds, st); }
}  // namespace wm
