// Persistent decode step, bf16_t plain weights, built for 1 row (one translation unit per
// instantiation set: they build in parallel)
#include "pdec_body.h"

namespace wm {
void pdec_launch_bf16_1(const PdecArgs& a, size_t lds, hipStream_t st) { pdec_launch_t<bf16_t, false, 1>(a, lds, st); }
}  // namespace wm
