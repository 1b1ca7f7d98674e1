// Host-side launchers of the gfx950 kernels. Every launcher takes the stream it runs on and
// never allocates or synchronises (so a decode step can be captured into a hipGraph).
#pragma once
#include <atomic>

#include "common.h"

namespace wm {

// ---- mel (kernels/mel.hip) ---------------------------------------------------------------------
void launch_mel(const float* const* d_pcm, const int* d_n, const void* d_tab, const float* d_filt_t, int n_mel,
                float* const* d_mel, const int* d_nlen, int* d_max, int n_jobs, int max_frames, hipStream_t st);
void launch_mel_window(DType dt, float* const* d_mel, const int* d_nlen, const int* d_n, const int* d_max,
                       const int* d_win_job, const int* d_win_seek, int n_win, int n_mel, void* out, hipStream_t st);
void launch_mel_normalize(const float* d_mel, int nl, int n_samples, const int* d_max, int n_mel, float* out, hipStream_t st);
// ---- audio front-end (kernels/audio.hip; audio.rs VAD chunking + resampler) ------------------------
// rms[c][w] (row stride rms_stride >= max_n / (rate/50)) of every 20 ms window, then per clip the
// noise floor (floor_out, optional) and the silence boundaries: counts[c], bounds[c][cap]
void launch_silence_boundaries(const float* const* pcm, const int* n_samples, int n_clips, int max_n, int sample_rate,
                               float* rms, int rms_stride, int* counts, int* bounds, int cap, float* floor_out,
                               hipStream_t st);
// out[c][m*fso + j] = sum_t in[c][(m-1)*fsi + t] * W[t][j] for m*fso + j < n_out[c]; W [2*fsi][ldw]
void launch_resample(const float* const* in, const int* n_in, int n_clips, int max_out, const float* W, int ldw, int fsi,
                     int fso, float* const* out, const int* n_out, hipStream_t st);

// ---- layer norm / embedding (kernels/norm.hip) ------------------------------------------------
// y[i] = LN(x[row(i)]) * w + b, x f32 [.][D] (row stride D), y T [M][D]; row(i) = rows ? rows[i] : i
void launch_layernorm(DType dt, const float* x, const int* rows, int M, int D, const float* w, const float* b,
                      void* y, hipStream_t st);
// x[i][:] = tok_emb[tok[i]][:] + pos_emb[pos[i]][:]   (f32 out; tok_emb in the MFMA type, or f32
// when te_f32: a quantized GGML embedding's exact dequantized rows)
void launch_embed(DType dt, const void* tok_emb, bool te_f32, const float* pos_emb, const int* tok, const int* pos,
                  int n, int D, float* x, hipStream_t st);
// embedding fused with the first LayerNorm: x as above, y[i] = LN(x[i]) * w + b (T out)
void launch_embed_ln(DType dt, const void* tok_emb, bool te_f32, const float* pos_emb, const int* tok, const int* pos,
                     int n, int D, float* x, const float* w, const float* b, void* y, hipStream_t st);

// ---- GEMM (kernels/gemm.hip): C[M][N] = A[M][K] . B[N][K]^T + bias, fused epilogues --------------
enum Epi : int {
    EPI_STORE = 0,     // T out[orow][n] = (v) * colscale(n)
    EPI_GELU = 1,      // T out = gelu_ggml(v)   (ggml's f16 GELU table)
    EPI_RESID = 2,     // f32 out[orow][n] = v + out[orow][n]            (residual stream, in place)
    EPI_GELU_POS = 3,  // f32 out = gelu_ggml(v) + pos[m % pos_rows][n]   (conv2 + positional emb)
    EPI_F32 = 4,       // f32 out = v                                       (logits)
    EPI_CROSSKV = 5,   // T scatter into cross cache [slot][L][2][H][ctx][64]; K columns scaled
    EPI_QKV_DEC = 6,   // n<d: T q[m][n]*scale ; d<=n<2d: K cache (scaled) ; 2d<=n<3d: V cache
    EPI_GELU_F = 7,    // T out = tanh-GELU by formula in f32 (fp8 mode, and bf16 encoders: not ggml's f16 table)
};

// GGML block-quantized weight matrix [N][K] (the app's catalog ships q5_0 / q5_1
// files, model.rs:153-186) kept in HBM as the file's blocks, regrouped by field (same bits, same bytes):
// qs = the quant bytes of every block [N][K/2] (q4_*, q5_*: two 4-bit values per byte, the block's
// weights j and j + 16 in byte j) or [N][K] (q8_0), qh = the q5 high bits [N][K/32] (bit j = weight j),
// dm = the f16 scale d per block [N][K/32] (q4_0, q5_0, q8_0) or d and min m [N][K/32][2] (q4_1,
// q5_1). type: ggml type id (2 q4_0, 3 q4_1,
// 6 q5_0, 7 q5_1, 8 q8_0), 0 = not quantized. w = d * (q - offset) or d * q + m, exact in f32, then
// rounded once to the compute type.
struct QMat {
    int type = 0;
    const uint8_t* qs = nullptr;
    const uint32_t* qh = nullptr;
    const uint16_t* dm = nullptr;
};

struct GemmArgs {
    const void* A; long a_rpb, a_bstride, a_rstride;  // A row m -> A + (m/a_rpb)*a_bstride + (m%a_rpb)*a_rstride
    const void* B;                                     // [N][K] row-major
    const float* bias;                                 // [N] or null
    int M, N, K;
    void* out; long ldo; long o_rpb, o_bstride, o_off; // out row = (m/o_rpb)*o_bstride + (m%o_rpb) + o_off
    const float* pos; int pos_rows;                    // EPI_GELU_POS
    float scale; int sc_div, sc_mod, sc_lim;           // column n scaled iff ((n/sc_div)%sc_mod) < sc_lim
    // caches (EPI_CROSSKV / EPI_QKV_DEC)
    void* cache; const int* row_slot; const int* row_pos; int L, layer, H, ctx, d;
    // split-K workspace for skinny (decode-step) GEMMs: f32 [splits][M][N]; null disables split-K
    float* splitk_ws; long splitk_ws_elems;
    // EPI_RESID on the split-K path only: fused LayerNorm of the updated residual rows,
    // ln_out[m][:] = LN(out[m][:]) * ln_w + ln_b (the next GEMM's input; null = no LN)
    const float* ln_w; const float* ln_b; void* ln_out;
    // small-M decode GEMM (launch_gemm_small) with lna: A is the f32 residual stream and the
    // workgroup applies LN(A) * a_ln_w + a_ln_b (ggml_norm) to its rows before the product
    const float* a_ln_w; const float* a_ln_b;
    // small-M decode GEMM: B given as GGML blocks (q.type != 0) instead of the compute type
    QMat q;
    // decode-step split-K slabs stored write-through (sc1) instead of write-back (every decode step)
    int slab_wt;
    // decode-step GEMMs in fp8 mode: B is OCP e4m3 [N][K] bytes, column n scaled by w8_scale[n]
    const float* w8_scale;
    // debug (whisper_mi355x_set_gemm_stamps): the encoder GEMM kernel writes s_memtime at 4 points per workgroup
    unsigned long long* stamps;
};
extern unsigned long long* g_gemm_stamps;

void launch_gemm(DType dt, int epi, const GemmArgs& a, hipStream_t st);
// fp8 (OCP e4m3) operands with per-row f32 scales: C = (A8 . B8^T) * a_scale[m] * b_scale[n], then
// the epilogue (EPI_STORE / EPI_GELU / EPI_GELU_F / EPI_RESID); K % 128 == 0, N % 16 == 0. A/B strides
// in bytes.
void launch_gemm_fp8(DType dt, int epi, const GemmArgs& a, const float* a_scale, const float* b_scale, hipStream_t st);
// q[r][:] = e4m3(x[r][:] / s[r]), s[r] = max|x[r][:]| / 448 (x in the MFMA type, K % 8 == 0)
void launch_quant_rows_fp8(DType dt, const void* x, long rows, int K, void* q, float* s, hipStream_t st);
// LayerNorm (f32 residual rows -> LN * w + b) quantized per row to fp8 e4m3: q [M][D] bytes, s [M]
void launch_layernorm_fp8(const float* x, int M, int D, const float* w, const float* b, void* q, float* s,
                          hipStream_t st);
// uploads the f16 GELU table the GELU epilogues read (once per context/device, before any GEMM)
void init_gelu_table();
// Decode step (M <= 128, K % 64 == 0): only the split-K partial sums, slabs [splits][M][N] f32 in
// a.splitk_ws, no epilogue; the consumer reduces them (attention prologues). Returns the split
// count, or 0 when the shape/workspace does not allow it (the caller then uses launch_gemm).
int launch_gemm_partials(DType dt, const GemmArgs& a, hipStream_t st);
// Decode steps of M <= 32 rows: one launch, no split-K slabs and no reduce launch (one workgroup =
// 16 output columns over the whole K, its 8 waves splitting K and summing in LDS). Epilogues
// EPI_F32 / EPI_STORE / EPI_GELU / EPI_RESID. lna: A = LN(f32 residual rows) computed in the
// prologue (K <= 1280). M > 32 runs as 32-row chunks (block-quantized weights, a.q, take this path at
// every batch size). gemm_small_ok: false when the shape is not supported (K % 32; lna: K <= 1280,
// K % 128).
bool gemm_small_ok(int M, int K, bool lna);
// out[r][k] (compute type) = the dequantized weights of rows [0, rows) of a block-quantized matrix
void launch_dequant(DType dt, const QMat& q, long rows, int K, void* out, hipStream_t st);
// up to 6 matrices of ONE GGML type dequantized by one launch (start[] is filled by the launcher)
struct DequantJobs {
    int n = 0;
    QMat q[6];
    long rows[6];
    int K[6];
    void* out[6];
    long start[7];
};
void launch_dequant_multi(DType dt, DequantJobs J, hipStream_t st);
void launch_gemm_small(DType dt, int epi, const GemmArgs& a, bool lna, hipStream_t st);

// ---- attention (kernels/attn.hip) --------------------------------------------------------------
// encoder self-attention: qkv [B*T][3d] -> out [B*T][d]; softmax scale 1/sqrt(64)
// variant: -1 = the default (6: attn_enc2_kernel held to 128 VGPRs, scalar softmax FMAs), else
// 1 / 2 / 3 / 5 (attn_enc_kernel / _enc2_ / _enc3_ / _enc2_ with packed FMAs; kernel benchmarks only)
void launch_attn_encoder(DType dt, const void* qkv, void* out, int B, int T, int d, int H, hipStream_t st,
                         int variant = -1);
// single-query attention for decoder tokens over a cache [slot][L][2][H][ctx][64]:
// token i attends keys [0, n_kv[i]) of slot[i]; q [n][q_stride] at head h offset h*64; out [n][d]
void launch_attn_decode(DType dt, const void* q, int q_stride, const void* cache, const int* slot, const int* n_kv,
                        int n, int L, int layer, int H, int ctx, int d, void* out, int kind, hipStream_t st);

// Prefill: the same attention for runs of consecutive tokens of one clip, tiles[t] = {first token,
// count <= 64} (int2), one workgroup per (tile, head); K/V staged once per tile.
void launch_attn_prefill(DType dt, const void* q, int q_stride, const void* cache, const int* slot, const int* n_kv,
                         const void* tiles, int n_tiles, int L, int layer, int H, int ctx, int d, void* out,
                         hipStream_t st);

// Decode-step attention with the projection GEMM's split-K reduce fused into its prologue.
// Slab z holds rows [M][ld] of partial sums; the value of (row i, column c) is
// sum_z ws[z*zstride + i*ld + c] + bias[c] (the same order as the standalone reduce).
struct DecSlabs {
    const float* ws; int splits; long zstride; int ld; const float* bias; float scale;
};
// self attention of token i: q/k/v columns [0,d)/[d,2d)/[2d,3d) of the QKV slabs (q and k scaled,
// as the EPI_QKV_DEC epilogue); writes this position's k, v into the self cache at pos[i].
void launch_attn_self_step(DType dt, const DecSlabs& sl, void* cache, const int* slot, const int* pos, int n, int L,
                           int layer, int H, int ctx, int d, void* out, hipStream_t st);
// decode steps of up to this many clips use the 1024-thread cache-form kernel (WHISPER_MI355X_XWIDE_MAX,
// default 4, read per call)
int attn_cross_wide_max();
// cross attention of token i over n_kv[i] keys of the cross cache; q from the cross-Q slabs.
void launch_attn_cross_step(DType dt, const DecSlabs& sl, const void* cache, const int* slot, const int* n_kv, int n,
                            int L, int layer, int H, int ctx, int d, void* out, hipStream_t st);

// ---- cross attention from the encoder output (kernels/xattn.hip) --------------------------------
// enc [slot][Tn][d] (the encoder's ln_post output in the MFMA type). For token i (clip slot[i]):
//   qproj:   qx[i][h][:] / qx[i][H+h][:] = hi / lo parts of scale * Wk_h^T q[i][h*64:(h+1)*64]
//            (wkt = Wk per head, transposed: [H][d][64]);
//   step:    rows split sp: unnormalised partial O^T opart[i][sp][h][d] and ml[i][sp][h] = {m (log2 units), l};
//            the running max moves only when a tile exceeds it by more than thr (log2 units);
//   combine: out[i][h*64+j] = (sum_sp w_sp O_sp / L) . Wv[h*64+j][:] + bv[h*64+j]   (MFMA type)
bool xattn_supported(int d);
int xattn_splits(int n, int Tn);
void launch_xattn_qproj(DType dt, const void* q, const void* wkt, int n, int d, int H, float scale, void* qx,
                        hipStream_t st);
void launch_xattn_step(DType dt, const void* enc, const int* slot, const void* qx, int n, int Tn, int d, int splits,
                       float thr, float* opart, float* ml, hipStream_t st);
void launch_xattn_combine(DType dt, const float* opart, const float* ml, int splits, const void* wv, const float* bv, int n,
                          int d, int H, void* out, hipStream_t st);

// ---- persistent decode step (kernels/pdec.hip) ---------------------------------------------------
// One launch = every decoder layer of one decode step for M <= kPdecMaxRows clips in the cross K/V cache
// form, phases handed off through data-tagged granules (see pdec.hip). Output: out_dh [M][d] (T) = the final
// LayerNorm of each row, the logits GEMM's input.
constexpr int kPdecMaxRows = 4;
// one projection matrix [N][K]: the compute type (qt = 0, w = T weights) or GGML blocks (qt = ggml type,
// w = QMat::qs, qh, dm as in QMat)
struct PdecMat {
    const void* w;
    const uint32_t* qh;
    const uint16_t* dm;
    int qt;
};
struct PdecLayer {
    PdecMat qkv, o, xq, xo, f1, f2;
    const float *bqkv, *bo, *bxq, *bxo, *b1, *b2;
    const float *ln1_w, *ln1_b, *lnx_w, *lnx_b, *ln2_w, *ln2_b;
};
// The hand-off block (one allocation, zeroed before every launch): data-tagged 8-byte granules (offsets
// in granules): x rows x0, x1, x2 [R][d] (f32), and packed T pairs: qkv [R][3d/2], self-attention output
// so [R][d/2], cross q qx [R][d/2], cross-attention output xo [R][d/2], GELU rows ff [R][2d]; the
// cross-attention split partials part [max(256, R * H * S)][66] (f32: o[64], max, sum; one per task); then the
// error word (byte offset); R = kPdecMaxRows.
struct PdecGranules {
    long x0, x1, x2, qkv, so, qx, xo, ff, part;
    long err_bytes, zero_bytes, bytes;  // the error word; 256 zero bytes that no one writes (a zero page)
};
PdecGranules pdec_granules(int d, int L, int H);
// LDS layout of one workgroup (byte offsets, 16-aligned), shared by the launcher and the kernel: rows are
// provisioned for the launch's clip count when it is 1 or 2 (those launches also hold the |x| < 10 part
// of ggml's f16 GELU table, 2 x 0x4900 entries), else for kPdecMaxRows
struct PdecLds {
    int xs, xf, sc, red, qf, res, ost, lred, lnp, part, lflag, gtab, bytes, rows, cmax;
};
constexpr int kPdecGeluHalf = 0x4900;  // f16 bit patterns below 10.0 (one sign)
__host__ __device__ inline PdecLds pdec_lds(int d, int M, int S) {
    auto up = [](int b) { return (b + 15) & ~15; };
    PdecLds l{};
    l.rows = M <= 2 ? M : kPdecMaxRows;
    const int c1 = 2 * ((3 * d / 2 + 255) / 256), c4 = 2 * ((2 * d + 255) / 256);
    l.cmax = c1 > c4 ? c1 : c4;
    int o = 0;
    l.xs = o; o += up(l.rows * 4 * d * 2);
    l.xf = o; o += up(l.rows * d * 4);
    l.sc = o; o += 1536 * 4;
    l.red = o; o += up((8 + 256) * 4);
    l.qf = o; o += 192 * 4;
    l.res = o; o += up(68 * 4);
    l.ost = o; o += up(l.rows * l.cmax * 4);
    l.lred = o; o += 2 * kPdecMaxRows * 4 * 8;
    l.lnp = o; o += up(6 * d * 4);
    l.part = o; o += up(S * 66 * 4);
    l.lflag = o; o += 16;
    l.gtab = o; o += M <= 2 ? up(2 * kPdecGeluHalf * 2) : 0;
    l.bytes = o;
    return l;
}
struct PdecArgs {
    const PdecLayer* layers;  // device array [L]
    int L, M, d, n_text_ctx, n_audio_ctx;
    const void* tok_emb; int te_f32; const float* pos_d;
    const float *lnd_w, *lnd_b;
    const int *tok, *pos, *slot;      // [M]
    void* self_cache; const void* cross_cache;
    float k_scale;
    int s_cross;                        // key splits per (clip, head) of the cross attention
    int quant;                          // the layers' matrices are GGML blocks (PdecMat.qt != 0)
    void* sync;                         // the hand-off block (gr.bytes), zeroed by the launcher
    PdecGranules gr;
    void* out_dh;
    const uint16_t* gelu_tab;           // ggml's f16 GELU table on the device (gelu_table_device)
    long spin_ticks;                    // a wait gives up after this many 100 MHz ticks (g_pdec_spin_ticks)
    unsigned long long* stamps;         // debug (g_pdec_stamps): [256][L][8][2] clock at input / publish, or null
};
extern unsigned long long* g_pdec_stamps;
// bumped by the stamps / spin setters: decode graphs captured with a persistent step under an older value
// are retired, not replayed (they hold the old pointer and limit as kernel arguments)
extern std::atomic<int> g_pdec_gen;  // bumped by the stamps / spin setters (capi.cpp); read once per dec_graph
// persistent launches that gave up, every state of the process (whisper_mi355x_pdec_give_ups(NULL))
extern std::atomic<long> g_pdec_give_ups_total;
// 5,000,000 = 50 ms; a test hook sets 0 to make every launch give up (the re-run path)
extern long g_pdec_spin_ticks;
// 1: quantized files' persistent steps stream the GGML blocks even when the expanded copy exists
extern int g_pdec_blocks;
// a kernel exists for the shape: plain weights at d 384 / 512 / 768 / 1024 / 1280, GGML blocks (f16
// compute) at 768 / 1024 / 1280
bool pdec_supported(int d, int H, bool quant);
int pdec_cross_splits(int H, int rows);  // key splits per (clip, head): a function of the shape only
void launch_pdec(DType dt, const PdecArgs& a, hipStream_t st);
const uint16_t* gelu_table_device();

// ---- logits processing (kernels/logits.hip) ----------------------------------------------------
struct VocabIds {
    int n_vocab, eot, sot, translate, transcribe, solm, prev, nosp, not_, beg, space, n_lang;
};
struct SeqCtl {             // per-sequence inputs of whisper_process_logits
    int is_initial, last_ts, penult_ts, has_ts, seek_delta;
    float temperature;
    int suppress_blank, no_timestamps, suppress_eot, tid0_initial;  // tid0_initial < 0: no max_initial_ts rule
    int want_probs, want_nosp;
};
struct TokOut { int id, tid; float p, plog, pt, ptsum, nosp_prob, pad; };
// rec: scratch of logits_rec_bytes(n_seq) bytes for the split form (rows spread over several workgroups
// each, used for up to 16 rows); null = one workgroup per row
void launch_logits(const float* logits, long ld, const SeqCtl* ctl, int n_seq, const VocabIds& v,
                   TokOut* out, float* probs, void* rec, hipStream_t st);
size_t logits_rec_bytes(int n_seq);
// pipelined greedy decoding: advance every row's input token, position and SeqCtl on the device after a step
// and copy its TokOut (+ the persistent launch's error word, if err) to a ring slot (kernels/logits.hip)
void launch_decode_advance(int n, int ct, int beg, const TokOut* tout, int* ints, SeqCtl* ctl, TokOut* ring,
                           const unsigned* err, unsigned* ring_err, hipStream_t st);

}  // namespace wm
