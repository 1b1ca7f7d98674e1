// TEST INFRASTRUCTURE ONLY — the CPU oracle for nobs-whisper_amd.
//
// This is a CPU restatement of the whisper.cpp algorithm that the reference app reaches through
// whisper-rs 0.15.1 / whisper-rs-sys 0.14.1 (src-tauri/Cargo.lock:5641-5659). whisper.cpp is a
// third-party dependency that is NOT present in /root/reference nor anywhere offline, so every
// function here restates the published algorithm of whisper.cpp ≈ v1.7.x from its source as
// published upstream ([ext] in SURVEY.md). Parity anchors: the reference's own call site and
// FullParams (src-tauri/src/whisper.rs:66-148), its post-filter tests (whisper.rs:285-305) and an
// independent implementation (HF transformers Whisper, local) used to pin mel + forward numerics
// (tests/golden/make_golden.py). The reference's whisper.cpp outputs themselves cannot be run
// here: for token IDs this oracle is "parity pinned to HF transformers, unpinned to whisper.cpp".
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code.
#pragma once
#include <cstdint>
#include <cstring>
#include <cmath>

namespace oracle {

// IEEE binary16 round-to-nearest-even, as ggml's GGML_FP32_TO_FP16 (F16C _cvtss_sh(x,0) or its
// software fallback ggml_compute_fp32_to_fp16) — [ext] ggml/src/ggml-impl.h.
static inline uint16_t f32_to_f16(float f) {
    uint32_t x; std::memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t mant = x & 0x007fffffu;
    int32_t exp = (int32_t)((x >> 23) & 0xff);
    if (exp == 0xff) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0));  // inf / nan
    int32_t e = exp - 127 + 15;
    if (e >= 0x1f) return (uint16_t)(sign | 0x7c00u);                         // overflow -> inf
    if (e <= 0) {                                                               // subnormal / zero
        if (e < -10) return (uint16_t)sign;
        mant |= 0x00800000u;
        const int shift = 14 - e;
        uint32_t h = mant >> shift;
        const uint32_t rem = mant & ((1u << shift) - 1);
        const uint32_t half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) h++;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)e << 10) | (mant >> 13);
    const uint32_t rem = mant & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;  // may carry into exponent: correct
    return (uint16_t)(sign | h);
}

static inline float f16_to_f32(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1f;
    uint32_t mant = h & 0x3ffu;
    uint32_t x;
    if (exp == 0) {
        if (mant == 0) { x = sign; }
        else {
            int e = -1;
            do { e++; mant <<= 1; } while (!(mant & 0x400u));
            mant &= 0x3ffu;
            x = sign | ((uint32_t)(127 - 15 - e) << 23) | (mant << 13);
        }
    } else if (exp == 0x1f) {
        x = sign | 0x7f800000u | (mant << 13);
    } else {
        x = sign | ((exp + 127 - 15) << 23) | (mant << 13);
    }
    float f; std::memcpy(&f, &x, 4); return f;
}

static inline float round_f16(float f) { return f16_to_f32(f32_to_f16(f)); }

}  // namespace oracle
