/*
 * whisper_mi355x.h — additive extensions of the whisper.h ABI for MI355X (SURVEY.md §8b
 * "Additive batch extension"). The reference calls one clip at a time
 * (src-tauri/src/whisper.rs:150-151: "GPU can only process one at a time"); these entry points
 * let a caller hand over many independent 30 s chunks at once, keep PCM resident in HBM, pick
 * the compute type, and broadcast weights to the other GPUs of a node over RCCL/xGMI.
 * Nothing here replaces a reference interface; whisper.h's functions are unchanged.
 */
#ifndef WHISPER_MI355X_H
#define WHISPER_MI355X_H

#include "whisper.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Return code of every entry point below (and of whisper_full_with_state / whisper_pcm_to_mel /
 * whisper_encode / whisper_decode) when the engine hit a device error (a HIP error such as out of
 * memory) or an unsupported shape: the call is abandoned, nothing is aborted, and the context and
 * the state stay usable (whisper.rs:127-129 maps any non-zero return to TranscriptionError). */
#define WHISPER_MI355X_ERR_RUNTIME (-10)

/* compute type of weights and GEMM activations. FP8_ENC: bf16, with the encoder's QKV, FC1 and FC2
 * GEMMs on OCP e4m3 weights and activations (per-row f32 scales; the large-v3-turbo fp8 config).
 * FP8_ENC is a throughput mode, not a whisper.cpp-parity mode. */
enum whisper_mi355x_dtype { WHISPER_MI355X_F16 = 0, WHISPER_MI355X_BF16 = 1, WHISPER_MI355X_FP8_ENC = 2 };

/* Context on HIP device `gpu_device` (from params) with an explicit compute type.
 * load_weights = false: parse the file and allocate the device weight arena without filling it
 * (a rank that receives the weights by whisper_mi355x_broadcast_weights). */
WHISPER_API struct whisper_context * whisper_mi355x_init(const char * path_model, struct whisper_context_params params,
                                                         int dtype, bool load_weights);

/* Device weight arena (one contiguous allocation holding every converted tensor). */
WHISPER_API int whisper_mi355x_weight_arena(struct whisper_context * ctx, void ** dev_ptr, size_t * bytes);

/* RCCL (rccl.h) unique id for a weight broadcast: filled by rank 0, shipped to the other ranks by
 * the caller (any side channel), then every rank calls whisper_mi355x_broadcast_weights. */
WHISPER_API int whisper_mi355x_rccl_unique_id(char out[128]);
WHISPER_API int whisper_mi355x_broadcast_weights(struct whisper_context * ctx, const char unique_id[128], int rank, int world);

/* Batched whisper_full: n_jobs independent clips, each processed exactly as one
 * whisper_full_with_state call on a fresh state would process it. pcm[j] points at n_samples[j]
 * f32 samples, on the host (pcm_on_device = false) or already in this context's HBM (true).
 * Fixed-work benchmark mode: fixed_tokens > 0 decodes exactly that many tokens per window with EOT
 * suppressed and no temperature fallback; at most n_text_ctx / 2 - 4 (a window's limit,
 * 220), else -1. Returns 0 on success. */
WHISPER_API int whisper_mi355x_full_batch(struct whisper_context * ctx, struct whisper_state * state,
                                          struct whisper_full_params params, const float * const * pcm,
                                          const int * n_samples, int n_jobs, bool pcm_on_device, int fixed_tokens);
/* Parity-test hook: the fixed-work batch with teacher forcing. The token decoded after step i of job j
 * is forced[j * fixed_tokens + i] (whatever the logits rules chose), and the raw logits of the jobs
 * spot[0..n_spot) at every step i (step 0 = the prefill) go to spot_logits[(i * n_spot + k) * n_vocab]
 * (host memory, fixed_tokens * n_spot * n_vocab floats). The kernels are the ones whisper_mi355x_full_batch
 * runs on the same batch (above 128 jobs: two concurrent halves, each forced and spot-copied by its own
 * jobs). */
WHISPER_API int whisper_mi355x_full_batch_forced(struct whisper_context * ctx, struct whisper_state * state,
                                                 struct whisper_full_params params, const float * const * pcm,
                                                 const int * n_samples, int n_jobs, bool pcm_on_device, int fixed_tokens,
                                                 const int * forced, const int * spot, int n_spot, float * spot_logits);
WHISPER_API int whisper_mi355x_batch_n_segments(struct whisper_state * state, int job);
WHISPER_API const char * whisper_mi355x_batch_segment_text(struct whisper_state * state, int job, int i_segment);
WHISPER_API int64_t whisper_mi355x_batch_segment_t0(struct whisper_state * state, int job, int i_segment);
WHISPER_API int64_t whisper_mi355x_batch_segment_t1(struct whisper_state * state, int job, int i_segment);
WHISPER_API int whisper_mi355x_batch_segment_n_tokens(struct whisper_state * state, int job, int i_segment);
WHISPER_API whisper_token_data whisper_mi355x_batch_token_data(struct whisper_state * state, int job, int i_segment, int i_token);
WHISPER_API int whisper_mi355x_batch_lang_id(struct whisper_state * state, int job);
/* tokens generated (all decode steps, all attempts) by the last whisper_mi355x_full_batch */
WHISPER_API long whisper_mi355x_batch_decoded_tokens(struct whisper_state * state);
/* tokens generated by every whisper_full / whisper_mi355x_full_batch call of the process so far (lets a
 * caller that drives whisper.h through its own states, e.g. the WhisperEngine mirror, count per call) */
WHISPER_API long whisper_mi355x_decoded_tokens_total(void);
/* Debug: the batched persistent decoder chain's hand-off counters and error word after the state's last
 * decode step (u32 words, out must hold them); returns the word count (-count if cap is too small). */
/* Debug: device pointers of a state's decode workspace (0 residual x, 1 final LayerNorm rows, 2 q|k|v rows of
 * the batched chain, 3 attention outputs, 4 GELU rows, 5 cross q, 6 Q', 7 cross-attention partials, 8 their
 * {m, l}); NULL when not allocated. */
WHISPER_API void * whisper_mi355x_debug_ws(struct whisper_state * state, int which);

/* Per-window decisions of whisper_full's temperature-fallback loop (the integer outcomes that are
 * comparable with whisper.cpp even when a sampled t > 0 attempt is not): one record per decoded
 * 30 s window, in seek order. temp_idx: index of the temperature finally used (0 = greedy t = 0
 * succeeded); n_attempts = temp_idx + 1; failed0: the t = 0 attempt failed (timestamp rule or
 * entropy < entropy_thold); logprob_fail0: its avg_logprob < logprob_thold; result_len0,
 * avg_logprob0, entropy0: that attempt's sequence score inputs; no_speech: the window was
 * dropped as silence. job = 0 for whisper_full_with_state. Returns the record count (or -count
 * when cap is too small). */
struct whisper_mi355x_window_decision {
    int32_t seek;
    int32_t temp_idx;
    int32_t failed0;
    int32_t logprob_fail0;
    int32_t result_len0;
    int32_t no_speech;
    float   avg_logprob0;
    float   entropy0;
    float   no_speech_prob;
    float   pad;
};
WHISPER_API int whisper_mi355x_window_decisions(struct whisper_state * state, int job,
                                                struct whisper_mi355x_window_decision * out, int cap);

/* Phase timings of the last full/full_batch call, milliseconds (host wall clock around
 * stream-synchronised phases): mel, encode (incl. cross-KV), prefill, decode steps, logits. */
WHISPER_API int whisper_mi355x_phase_ms(struct whisper_state * state, double out[5]);

/* Normalised log-mel of the last whisper_pcm_to_mel_with_state / whisper_full_with_state call,
 * copied to host: [n_mel][n_len] f32. Returns n_len. */
WHISPER_API int whisper_mi355x_get_mel(struct whisper_state * state, float * out, int cap_floats);
/* Encoder output (ln_post) of window 0 of the last encode, [n_audio_ctx][n_audio_state] f32. */
WHISPER_API int whisper_mi355x_get_encoder_out(struct whisper_state * state, float * out, int cap_floats);

/* Live per-kernel-class timing with HIP events on the state's stream (used by bench.py for the
 * roofline). Classes: 0 encoder-side GEMM (work = FLOPs), 1 encoder attention (FLOPs),
 * 2 decoder cross-attention (HBM bytes), 3 decoder self-attention (bytes), 4 decoder GEMM (bytes),
 * 5 logits processing (bytes), 6 mel (bytes), 7 the persistent decode step (bytes), 8 the batched
 * persistent decoder chain (bytes). class_mask bit k times class k (0 = off); bits 16..23, when > 1, time
 * the decoder's per-layer attention launches (classes 2, 3) of every k-th layer only.
 * Every call resets the counters; stats out = {total ms, launches, total work}. */
WHISPER_API int whisper_mi355x_kernel_timing(struct whisper_state * state, int class_mask);
WHISPER_API int whisper_mi355x_kernel_stats(struct whisper_state * state, int cls, double out[3]);
/* Pseudo class of whisper_mi355x_kernel_stats: out = {ms lost, give-ups, 0} of the persistent decode step
 * (kernels/pdec.hip) on this state since it was created (or recycled): a launch that gave up (not all of its
 * 256 workgroups became resident within the wait limit, e.g. another process held CUs) is re-run on the
 * per-kernel path, and the state's next steps take that path for about a second. Not reset by
 * whisper_mi355x_kernel_timing. whisper_mi355x_pdec_give_ups returns the count alone (NULL: the total of every
 * state of the process). */
#define WHISPER_MI355X_KSTAT_PDEC_GIVE_UPS 100
WHISPER_API long whisper_mi355x_pdec_give_ups(struct whisper_state * state);

/* Kernel-level test/tuning hooks (device pointers): one fused-epilogue GEMM launch of the engine
 * (epi as in kernels.h: 0 store, 1 gelu, 2 residual f32, 4 f32, 5 cross K/V: out is then a cross cache of
 * M / n_audio_ctx slots for N / 2K layers, K = d), averaged over reps; and the
 * GEMM variant override (-1 auto, 0 register-staged, 1 LDS-DMA). */
WHISPER_API int whisper_mi355x_debug_gemm(struct whisper_context * ctx, int epi, const void * A, int M, int K,
                                          const void * B, int N, const float * bias, void * out, int reps, float * ms);
WHISPER_API void whisper_mi355x_set_gemm_variant(int variant);
/* debug: device buffer of [grid][4] u64 the encoder GEMM kernel fills with s_memtime stamps (entry, main loop
 * start / end, epilogue end) per workgroup; null turns it off */
WHISPER_API void whisper_mi355x_set_gemm_stamps(void * dev);
/* Debug/tuning: the small-M decode GEMM (M <= 32, K % 256 == 0): out = A.B^T + bias with epilogue epi
 * (2 residual: out f32 += ..., 4 f32, 0 store, 1 gelu); with ln_w != NULL, A is f32 [M][K] and the
 * product uses LN(A) * ln_w + ln_b (K <= 1280). The first launch's result stays in out; reps more
 * launches are timed (note: epi 2 accumulates into out on every launch). */
WHISPER_API int whisper_mi355x_debug_gemm_small(struct whisper_context * ctx, int epi, const void * A, int M, int K,
                                                const void * B, int N, const float * bias, void * out,
                                                const float * ln_w, const float * ln_b, int reps, float * ms);
WHISPER_API void whisper_mi355x_set_dec_splits(int splits); /* 0 = heuristic */
/* Test hook: the split-K decode GEMM's smallest row tile (32, 64 or 128; 0 = WHISPER_MI355X_DEC_BM or 32).
 * A step takes the smallest tile holding its rows; every value gives the same bits. */
WHISPER_API void whisper_mi355x_set_dec_bm(int rows);
/* Test hook: a persistent decode step's waits give up after this many 100 MHz ticks (default 5,000,000 =
 * 50 ms); 0 makes every persistent launch give up, so each step takes the re-run path. Decode graphs
 * captured before the call are retired (not replayed) once it changes the value; likewise for the stamps
 * pointer below, so a freed stamps buffer is never written. */
WHISPER_API void whisper_mi355x_set_pdec_spin(long ticks);
/* Profiling hook: device buffer of 256 * n_text_layer * 8 * 2 u64 that persistent decode steps captured
 * from now on fill with the 100 MHz clock (per workgroup, layer and phase: input arrived, phase
 * signalled); NULL turns it off. */
WHISPER_API void whisper_mi355x_set_pdec_stamps(void * dev);
/* Quantized files: 1 = persistent decode steps stream the GGML blocks; 0 (default) = they read the
 * context's expanded compute-type copy once it exists (faster). */
WHISPER_API void whisper_mi355x_set_pdec_blocks(int on);
/* Debug/tuning: the decode-step residual GEMM with its fused LayerNorm (M <= 128):
 * x[M][N] (f32, in/out) += A.B^T + bias, then y[M][N] (compute dtype) = LN(x) * ln_w + ln_b. */
// fp8 (OCP e4m3) GEMM with per-row f32 scales (A per row m, B per row n), then epilogue `epi`;
// A8 [M][K], B8 [N][K] bytes, K % 128 == 0 (large-v3-turbo fp8 encoder path)
WHISPER_API int whisper_mi355x_debug_gemm_fp8(struct whisper_context * ctx, int epi, const void * A8,
                                              const float * a_scale, int M, int K, const void * B8,
                                              const float * b_scale, int N, const float * bias, void * out,
                                              int reps, float * ms);
// decode-step GEMM with e4m3 weights (fp8 mode decoder): out = A[M][K] (compute dtype) .
// (B8[N][K] e4m3 * b_scale[n])^T + bias, epilogue `epi`, M <= 128, K % 64 == 0; with epi 2 and
// ln_w != null the fused residual + LayerNorm form (x = out in/out, y = LN output)
WHISPER_API int whisper_mi355x_debug_gemm_w8(struct whisper_context * ctx, int epi, const void * A, int M, int K,
                                             const void * B8, const float * b_scale, int N, const float * bias,
                                             void * out, const float * ln_w, const float * ln_b, void * y);
// q[r][:] = e4m3(x[r][:] / s[r]), s[r] = max|x[r][:]| / 448; x in the context's MFMA type
WHISPER_API int whisper_mi355x_debug_quant_fp8(struct whisper_context * ctx, const void * x, long rows, int K,
                                               void * q, float * s);
/* Debug/tuning: one encoder self-attention launch (device pointers): qkv [B*T][3d] (Q | K | V, compute
 * type of ctx), out [B*T][d]; variant 1 / 2 / 3 / 5 = attn_enc_kernel / attn_enc2_kernel / attn_enc3_kernel /
 * attn_enc2_kernel held to 128 VGPRs, two workgroups per CU (d = 64 H). The first launch's result stays in out; reps more launches are timed (ms per launch). */
WHISPER_API int whisper_mi355x_debug_attn_encoder(struct whisper_context * ctx, const void * qkv, int B, int T, int d,
                                                  int H, int variant, void * out, int reps, float * ms);
WHISPER_API int whisper_mi355x_debug_gemm_ln(struct whisper_context * ctx, const void * A, int M, int K,
                                             const void * B, int N, const float * bias, float * x,
                                             const float * ln_w, const float * ln_b, void * y, int reps, float * ms);

/* Debug/tuning: the direct cross attention of decode steps (Q' projection, one pass over the
 * encoder output per token, split merge + value projection) on caller data, device pointers in the
 * context's compute type: enc [slots][n_ctx][d], slot [n] (int), q [n][d] (already scaled by
 * d_head^-0.25), wkt [d/64][d][64] (cross K weights per head, transposed), wv [d][d], bv [d] (f32)
 * -> out [n][d]. splits <= 0 picks the engine's split count; rescale_thr is the online-softmax
 * lazy-rescale threshold in log2 units (the engine uses 8). */
WHISPER_API int whisper_mi355x_debug_xattn(struct whisper_context * ctx, const void * enc, const int * slot,
                                           const void * q, const void * wkt, const void * wv, const float * bv,
                                           int n, int n_ctx, int d, float scale, int splits, float rescale_thr,
                                           void * out, int reps, float * ms);

/* Audio front-end on the GPU (src-tauri/src/audio.rs), for n_clips clips at
 * once on HIP device `device`. pcm / audio / out point at host buffers, or (on_device = true) at
 * buffers already in that device's HBM.
 *
 * whisper_mi355x_find_silence_boundaries replaces audio.rs:400-467 find_silence_boundaries(audio,
 * sample_rate) (with estimate_noise_floor, audio.rs:373-397): counts[c] = number of split points of
 * clip c (only the first `cap` are stored, boundaries[c * cap + i], sample indices); noise_floor[c]
 * (optional) = the adaptive noise floor; rms_out (optional, [n_clips][rms_stride]) = the RMS of
 * every 20 ms window, bit-identical to audio.rs:364-370 calculate_rms. Returns 0, or -1 on bad
 * arguments. split_at_silences (audio.rs:469-507) is pure indexing and stays with the caller. */
WHISPER_API int whisper_mi355x_find_silence_boundaries(int device, const float * const * pcm, const int * n_samples,
                                                       int n_clips, int sample_rate, bool pcm_on_device, int * counts,
                                                       int * boundaries, int cap, float * noise_floor, float * rms_out,
                                                       int rms_stride);
/* audio.rs:331-337 resample_chunk(audio, input_sample_rate) -> 16 kHz (audio.rs:509-563: rubato 0.15.0
 * FftFixedIn, 1024-sample chunks, 2 sub-chunks, last chunk zero-padded, output truncated to
 * len * 16000 / rate). out[c] must hold whisper_mi355x_resample_len(n_in[c], rate_in) floats. */
WHISPER_API int whisper_mi355x_resample_len(int n_in, int rate_in);
WHISPER_API int whisper_mi355x_resample_chunk(int device, const float * const * audio, const int * n_in, int n_clips,
                                              int rate_in, bool on_device, float * const * out);
/* The resampler's FFT pipeline as one linear map (tests): block sizes fsi / fso of rate_in, and
 * W [2*fsi][fso] with output block m = sum_t x[(m-1)*fsi + t] W[t][:]. */
WHISPER_API int whisper_mi355x_resample_operator(int rate_in, int * fsi, int * fso, float * W, long cap);

/* ABI self-description, no device needed: sizeof(whisper_full_params), sizeof(whisper_context_params),
 * sizeof(whisper_token_data), offsetof(full_params, initial_prompt / language / greedy /
 * new_segment_callback / vad_params). Lets a binding (bindgen, ctypes) be checked field-by-field. */
WHISPER_API int whisper_mi355x_abi_layout(size_t out[8]);

/* State introspection (tests): out[0] = cross-attention form of the last call (1 = straight from the
 * encoder output, 0 = cached cross K/V), out[1] = clip slots of the workspace, out[2] = slots of the
 * cross K/V cache, out[3] = decode-step graphs kept, out[4] = 1 if the state was recycled from the
 * context's state pool (whisper_init_state after a whisper_free_state keeps the workspace and the
 * captured decode graphs; WHISPER_MI355X_STATE_POOL=0 disables the pool). Returns 5. */
WHISPER_API int whisper_mi355x_state_info(struct whisper_state * state, int out[5]);

/* HIP stream of a state (hipStream_t), for callers that enqueue their own work around it. */
WHISPER_API void * whisper_mi355x_state_stream(struct whisper_state * state);

/* Model-free micro-API used by the kernel parity tests: allocate/copy device memory on the
 * context's device. */
WHISPER_API void * whisper_mi355x_dev_alloc(struct whisper_context * ctx, size_t bytes);
WHISPER_API void   whisper_mi355x_dev_free(struct whisper_context * ctx, void * p);
WHISPER_API int    whisper_mi355x_memcpy(struct whisper_context * ctx, void * dst, const void * src, size_t bytes, int kind);

#ifdef __cplusplus
}
#endif

#endif /* WHISPER_MI355X_H */
