// Persistent decode step, half_t plain weights, built for 4 rows (one translation unit per
// instantiation set: they build in parallel)
#include "pdec_body.h"

namespace wm {
void pdec_launch_f16_4(const PdecArgs& a, size_t lds, hipStream_t st) { pdec_launch_t<half_t, false, 4>(a, lds, st); }
}  // namespace wm
