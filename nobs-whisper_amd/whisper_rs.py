"""ctypes binding of libwhisper_mi355x.so shaped like the whisper-rs 0.15.1 API the reference uses
(src-tauri/src/whisper.rs:3): WhisperContextParameters, WhisperContext.new_with_params,
create_state, FullParams, SamplingStrategy.Greedy, WhisperState.full / full_n_segments /
get_segment. Python is plumbing here (tests, bench.py); the product is the C ABI + HIP kernels.

Loading fails loudly if the shared library is missing: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref
from dataclasses import dataclass

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WHISPER_MI355X_LIB") or os.path.join(HERE, "lib", "libwhisper_mi355x.so")  # override: A/B of two builds
ENGINE_LIB_PATH = os.path.join(HERE, "lib", "libnobs_whisper_engine.so")

# The app's default custom vocabulary (src-tauri/src/config.rs:40-42): the initial prompt of every
# transcribe call (whisper.rs:98-109, state.rs:276-279) unless the user edits the config file.
DEFAULT_VOCABULARY = (
    "Claude Code, Anthropic, Supabase, Vercel, shadcn, tRPC, Drizzle, Zod, pnpm, Bun, Deno, Turso, Neon, "
    "PlanetScale, Turborepo, Tauri, SvelteKit, Nuxt, Astro, Vite, Zustand, TanStack, LangChain, LlamaIndex, "
    "Ollama, Cursor, Neovim, Vitest, Playwright, Prisma, Radix, Fly.io, Railway, Cloudflare Workers, Hono, htmx, "
    "Biome, oxlint, Rspack, Turbopack, Qwik, SolidJS, Convex, Upstash, Resend, Inngest, Replit, v0, Lovable, Bolt, "
    "WindSurf, Codeium, Supermaven, Aider, OpenRouter, Perplexity, Groq, Mistral, Cohere, Replicate")

F16, BF16 = 0, 1
FP8_ENC = 2  # bf16 with the encoder QKV/FC1/FC2 GEMMs in fp8 e4m3 (large-v3-turbo fp8 config)
GREEDY, BEAM_SEARCH = 0, 1


class WhisperAheads(C.Structure):
    _fields_ = [("n_heads", C.c_size_t), ("heads", C.c_void_p)]


class WhisperContextParams(C.Structure):
    _fields_ = [("use_gpu", C.c_bool), ("flash_attn", C.c_bool), ("gpu_device", C.c_int),
                ("dtw_token_timestamps", C.c_bool), ("dtw_aheads_preset", C.c_int), ("dtw_n_top", C.c_int),
                ("dtw_aheads", WhisperAheads), ("dtw_mem_size", C.c_size_t)]


class _Greedy(C.Structure):
    _fields_ = [("best_of", C.c_int)]


class _Beam(C.Structure):
    _fields_ = [("beam_size", C.c_int), ("patience", C.c_float)]


class VadParams(C.Structure):
    _fields_ = [("threshold", C.c_float), ("min_speech_duration_ms", C.c_int), ("min_silence_duration_ms", C.c_int),
                ("max_speech_duration_s", C.c_float), ("speech_pad_ms", C.c_int), ("samples_overlap", C.c_float)]


class FullParams(C.Structure):
    """struct whisper_full_params (include/whisper.h), field for field."""
    _fields_ = [
        ("strategy", C.c_int), ("n_threads", C.c_int), ("n_max_text_ctx", C.c_int), ("offset_ms", C.c_int),
        ("duration_ms", C.c_int),
        ("translate", C.c_bool), ("no_context", C.c_bool), ("no_timestamps", C.c_bool), ("single_segment", C.c_bool),
        ("print_special", C.c_bool), ("print_progress", C.c_bool), ("print_realtime", C.c_bool),
        ("print_timestamps", C.c_bool),
        ("token_timestamps", C.c_bool), ("thold_pt", C.c_float), ("thold_ptsum", C.c_float), ("max_len", C.c_int),
        ("split_on_word", C.c_bool), ("max_tokens", C.c_int),
        ("debug_mode", C.c_bool), ("audio_ctx", C.c_int),
        ("tdrz_enable", C.c_bool),
        ("suppress_regex", C.c_char_p),
        ("initial_prompt", C.c_char_p), ("prompt_tokens", C.c_void_p), ("prompt_n_tokens", C.c_int),
        ("language", C.c_char_p), ("detect_language", C.c_bool),
        ("suppress_blank", C.c_bool), ("suppress_nst", C.c_bool),
        ("temperature", C.c_float), ("max_initial_ts", C.c_float), ("length_penalty", C.c_float),
        ("temperature_inc", C.c_float), ("entropy_thold", C.c_float), ("logprob_thold", C.c_float),
        ("no_speech_thold", C.c_float),
        ("greedy", _Greedy), ("beam_search", _Beam),
        ("new_segment_callback", C.c_void_p), ("new_segment_callback_user_data", C.c_void_p),
        ("progress_callback", C.c_void_p), ("progress_callback_user_data", C.c_void_p),
        ("encoder_begin_callback", C.c_void_p), ("encoder_begin_callback_user_data", C.c_void_p),
        ("abort_callback", C.c_void_p), ("abort_callback_user_data", C.c_void_p),
        ("logits_filter_callback", C.c_void_p), ("logits_filter_callback_user_data", C.c_void_p),
        ("grammar_rules", C.c_void_p), ("n_grammar_rules", C.c_size_t), ("i_start_rule", C.c_size_t),
        ("grammar_penalty", C.c_float),
        ("vad", C.c_bool), ("vad_model_path", C.c_char_p), ("vad_params", VadParams),
    ]


class TokenData(C.Structure):
    _fields_ = [("id", C.c_int32), ("tid", C.c_int32), ("p", C.c_float), ("plog", C.c_float), ("pt", C.c_float),
                ("ptsum", C.c_float), ("t0", C.c_int64), ("t1", C.c_int64), ("t_dtw", C.c_int64), ("vlen", C.c_float)]


class WindowDecision(C.Structure):
    """struct whisper_mi355x_window_decision (include/whisper_mi355x.h)."""
    _fields_ = [("seek", C.c_int32), ("temp_idx", C.c_int32), ("failed0", C.c_int32), ("logprob_fail0", C.c_int32),
                ("result_len0", C.c_int32), ("no_speech", C.c_int32), ("avg_logprob0", C.c_float),
                ("entropy0", C.c_float), ("no_speech_prob", C.c_float), ("pad", C.c_float)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C nobs-whisper_amd` (no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    vp, ip, fp = C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_float)
    sig = {
        "whisper_context_default_params": (WhisperContextParams, []),
        "whisper_full_default_params": (FullParams, [C.c_int]),
        "whisper_init_from_file_with_params_no_state": (vp, [C.c_char_p, WhisperContextParams]),
        "whisper_mi355x_init": (vp, [C.c_char_p, WhisperContextParams, C.c_int, C.c_bool]),
        "whisper_init_state": (vp, [vp]),
        "whisper_free": (None, [vp]),
        "whisper_free_state": (None, [vp]),
        "whisper_full_with_state": (C.c_int, [vp, vp, FullParams, fp, C.c_int]),
        "whisper_full_n_segments_from_state": (C.c_int, [vp]),
        "whisper_full_get_segment_text_from_state": (C.c_char_p, [vp, C.c_int]),
        "whisper_full_get_segment_t0_from_state": (C.c_int64, [vp, C.c_int]),
        "whisper_full_get_segment_t1_from_state": (C.c_int64, [vp, C.c_int]),
        "whisper_full_n_tokens_from_state": (C.c_int, [vp, C.c_int]),
        "whisper_full_get_token_data_from_state": (TokenData, [vp, C.c_int, C.c_int]),
        "whisper_full_get_segment_no_speech_prob_from_state": (C.c_float, [vp, C.c_int]),
        "whisper_full_lang_id_from_state": (C.c_int, [vp]),
        "whisper_pcm_to_mel_with_state": (C.c_int, [vp, vp, fp, C.c_int, C.c_int]),
        "whisper_encode_with_state": (C.c_int, [vp, vp, C.c_int, C.c_int]),
        "whisper_decode_with_state": (C.c_int, [vp, vp, ip, C.c_int, C.c_int, C.c_int]),
        "whisper_get_logits_from_state": (fp, [vp]),
        "whisper_tokenize": (C.c_int, [vp, C.c_char_p, ip, C.c_int]),
        "whisper_lang_auto_detect_with_state": (C.c_int, [vp, vp, C.c_int, C.c_int, fp]),
        "whisper_n_vocab": (C.c_int, [vp]),
        "whisper_is_multilingual": (C.c_int, [vp]),
        "whisper_model_n_vocab": (C.c_int, [vp]),
        "whisper_model_n_audio_state": (C.c_int, [vp]),
        "whisper_model_n_audio_layer": (C.c_int, [vp]),
        "whisper_model_n_text_layer": (C.c_int, [vp]),
        "whisper_model_n_mels": (C.c_int, [vp]),
        "whisper_token_sot": (C.c_int, [vp]),
        "whisper_token_eot": (C.c_int, [vp]),
        "whisper_token_beg": (C.c_int, [vp]),
        "whisper_token_transcribe": (C.c_int, [vp]),
        "whisper_token_to_str": (C.c_char_p, [vp, C.c_int]),
        "whisper_lang_id": (C.c_int, [C.c_char_p]),
        "whisper_lang_str": (C.c_char_p, [C.c_int]),
        "whisper_mi355x_full_batch": (C.c_int, [vp, vp, FullParams, C.POINTER(vp), ip, C.c_int, C.c_bool, C.c_int]),
        "whisper_mi355x_full_batch_forced": (C.c_int, [vp, vp, FullParams, C.POINTER(vp), ip, C.c_int, C.c_bool, C.c_int,
                                                       ip, ip, C.c_int, C.POINTER(C.c_float)]),
        "whisper_mi355x_batch_n_segments": (C.c_int, [vp, C.c_int]),
        "whisper_mi355x_batch_segment_text": (C.c_char_p, [vp, C.c_int, C.c_int]),
        "whisper_mi355x_batch_segment_t0": (C.c_int64, [vp, C.c_int, C.c_int]),
        "whisper_mi355x_batch_segment_t1": (C.c_int64, [vp, C.c_int, C.c_int]),
        "whisper_mi355x_batch_segment_n_tokens": (C.c_int, [vp, C.c_int, C.c_int]),
        "whisper_mi355x_batch_token_data": (TokenData, [vp, C.c_int, C.c_int, C.c_int]),
        "whisper_mi355x_batch_lang_id": (C.c_int, [vp, C.c_int]),
        "whisper_mi355x_batch_decoded_tokens": (C.c_long, [vp]),
        "whisper_mi355x_window_decisions": (C.c_int, [vp, C.c_int, C.POINTER(WindowDecision), C.c_int]),
        "whisper_mi355x_phase_ms": (C.c_int, [vp, C.POINTER(C.c_double)]),
        "whisper_mi355x_get_mel": (C.c_int, [vp, fp, C.c_int]),
        "whisper_mi355x_get_encoder_out": (C.c_int, [vp, fp, C.c_int]),
        "whisper_mi355x_state_stream": (vp, [vp]),
        "whisper_mi355x_state_info": (C.c_int, [vp, ip]),
        "whisper_mi355x_weight_arena": (C.c_int, [vp, C.POINTER(vp), C.POINTER(C.c_size_t)]),
        "whisper_mi355x_rccl_unique_id": (C.c_int, [C.c_char_p]),
        "whisper_mi355x_broadcast_weights": (C.c_int, [vp, C.c_char_p, C.c_int, C.c_int]),
        "whisper_mi355x_dev_alloc": (vp, [vp, C.c_size_t]),
        "whisper_mi355x_dev_free": (None, [vp, vp]),
        "whisper_mi355x_memcpy": (C.c_int, [vp, vp, vp, C.c_size_t, C.c_int]),
        "whisper_mi355x_abi_layout": (C.c_int, [C.POINTER(C.c_size_t)]),
        "whisper_mi355x_kernel_timing": (C.c_int, [vp, C.c_int]),
        "whisper_mi355x_kernel_stats": (C.c_int, [vp, C.c_int, C.POINTER(C.c_double)]),
        "whisper_mi355x_pdec_give_ups": (C.c_long, [vp]),
        "whisper_mi355x_decoded_tokens_total": (C.c_long, []),
        "whisper_mi355x_debug_ws": (vp, [vp, C.c_int]),
        "whisper_mi355x_set_pdec_spin": (None, [C.c_long]),
        "whisper_mi355x_set_pdec_stamps": (None, [vp]),
        "whisper_mi355x_set_gemm_stamps": (None, [vp]),
        "whisper_mi355x_set_pdec_blocks": (None, [C.c_int]),
        "whisper_mi355x_find_silence_boundaries": (C.c_int, [C.c_int, C.POINTER(vp), ip, C.c_int, C.c_int, C.c_bool,
                                                             ip, ip, C.c_int, fp, fp, C.c_int]),
        "whisper_mi355x_resample_len": (C.c_int, [C.c_int, C.c_int]),
        "whisper_mi355x_resample_chunk": (C.c_int, [C.c_int, C.POINTER(vp), ip, C.c_int, C.c_int, C.c_bool,
                                                    C.POINTER(vp)]),
        "whisper_mi355x_resample_operator": (C.c_int, [C.c_int, ip, ip, fp, C.c_long]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


# ---- whisper-rs shaped API ---------------------------------------------------------------------
@dataclass
class Segment:
    t0: int
    t1: int
    text: bytes
    tokens: list


def reference_full_params(language: str | None = "en", initial_prompt: str | None = None) -> FullParams:
    """FullParams::new(Greedy{best_of: 1}) + the setters of src-tauri/src/whisper.rs:91-124."""
    p = lib().whisper_full_default_params(GREEDY)
    p.greedy.best_of = 1
    p.language = language.encode() if language else None
    p.initial_prompt = initial_prompt.encode() if initial_prompt else None
    p.print_special = False
    p.print_progress = False
    p.print_realtime = False
    p.print_timestamps = False
    p.translate = False
    p.no_context = False
    p.single_segment = False
    p.suppress_blank = True
    p.no_speech_thold = 0.6
    p.entropy_thold = 2.4
    p.logprob_thold = -1.0
    return p


class WhisperContext:
    def __init__(self, path: str, dtype: int = F16, gpu_device: int = 0, load_weights: bool = True):
        L = lib()
        cp = L.whisper_context_default_params()
        cp.use_gpu = True
        cp.gpu_device = gpu_device
        self.L = L
        self.gpu_device = gpu_device
        self._states = weakref.WeakSet()
        self.ptr = L.whisper_mi355x_init(path.encode(), cp, dtype, load_weights)
        if not self.ptr:
            raise RuntimeError(f"whisper_mi355x_init failed for {path}")

    @classmethod
    def new_with_params(cls, path: str, use_gpu: bool = True):
        """WhisperContext::new_with_params (whisper.rs:41-45): the plain whisper.h entry point."""
        self = cls.__new__(cls)
        L = lib()
        cp = L.whisper_context_default_params()
        cp.use_gpu = use_gpu
        self.L = L
        self.gpu_device = cp.gpu_device
        self._states = weakref.WeakSet()
        self.ptr = L.whisper_init_from_file_with_params_no_state(path.encode(), cp)
        if not self.ptr:
            raise RuntimeError(f"failed to load {path}")
        return self

    def create_state(self) -> "WhisperState":
        return WhisperState(self)

    def tokenize(self, text: str) -> list:
        buf = (C.c_int * 4096)()
        n = self.L.whisper_tokenize(self.ptr, text.encode(), buf, 4096)
        return list(buf[:n])

    def close(self):
        # states first, as whisper.h requires (a garbage collector may finalise a context and its
        # states in any order; the library also tolerates the reverse order)
        for st in list(getattr(self, "_states", ())):
            st.close()
        if self.ptr:
            self.L.whisper_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class WhisperState:
    def __init__(self, ctx: WhisperContext):
        self.ctx = ctx
        self.L = ctx.L
        self.ptr = self.L.whisper_init_state(ctx.ptr)
        if not self.ptr:
            raise RuntimeError("whisper_init_state failed")
        ctx._states.add(self)

    def full(self, params: FullParams, audio) -> int:
        import numpy as np
        a = np.ascontiguousarray(audio, dtype=np.float32)
        return self.L.whisper_full_with_state(self.ctx.ptr, self.ptr, params,
                                              a.ctypes.data_as(C.POINTER(C.c_float)), len(a))

    def full_n_segments(self) -> int:
        return self.L.whisper_full_n_segments_from_state(self.ptr)

    def get_segment(self, i: int) -> Segment:
        L = self.L
        toks = []
        for t in range(L.whisper_full_n_tokens_from_state(self.ptr, i)):
            d = L.whisper_full_get_token_data_from_state(self.ptr, i, t)
            toks.append((d.id, d.tid, d.p, d.plog))
        return Segment(L.whisper_full_get_segment_t0_from_state(self.ptr, i),
                       L.whisper_full_get_segment_t1_from_state(self.ptr, i),
                       L.whisper_full_get_segment_text_from_state(self.ptr, i), toks)

    def segments(self) -> list:
        return [self.get_segment(i) for i in range(self.full_n_segments())]

    def full_batch(self, params: FullParams, pcm_list, on_device: bool = False, fixed_tokens: int = 0) -> int:
        """whisper_mi355x_full_batch. pcm_list: numpy arrays (host) or device pointers (ints)."""
        import numpy as np
        n = len(pcm_list)
        ptrs = (C.c_void_p * n)()
        lens = (C.c_int * n)()
        keep = []
        for i, x in enumerate(pcm_list):
            if on_device:
                ptrs[i], lens[i] = x[0], x[1]
            else:
                a = np.ascontiguousarray(x, dtype=np.float32)
                keep.append(a)
                ptrs[i] = a.ctypes.data
                lens[i] = len(a)
        return self.L.whisper_mi355x_full_batch(self.ctx.ptr, self.ptr, params, ptrs, lens, n, on_device, fixed_tokens)

    def full_batch_forced(self, params: FullParams, pcm_list, fixed_tokens: int, forced, spot, n_vocab: int,
                          on_device: bool = False):
        """whisper_mi355x_full_batch_forced: forced [n_jobs][fixed_tokens] token ids; returns (rc, logits
        [fixed_tokens][len(spot)][n_vocab]) of the spot jobs at every step."""
        import numpy as np
        n = len(pcm_list)
        ptrs = (C.c_void_p * n)()
        lens = (C.c_int * n)()
        keep = []
        for i, x in enumerate(pcm_list):
            if on_device:
                ptrs[i], lens[i] = x[0], x[1]
            else:
                a = np.ascontiguousarray(x, dtype=np.float32)
                keep.append(a)
                ptrs[i] = a.ctypes.data
                lens[i] = len(a)
        f = np.ascontiguousarray(forced, dtype=np.int32).reshape(n, fixed_tokens)
        sp = np.ascontiguousarray(spot, dtype=np.int32)
        out = np.zeros((fixed_tokens, len(sp), n_vocab), np.float32)
        ip_ = C.POINTER(C.c_int)
        rc = self.L.whisper_mi355x_full_batch_forced(self.ctx.ptr, self.ptr, params, ptrs, lens, n, on_device, fixed_tokens,
                                                     f.ctypes.data_as(ip_), sp.ctypes.data_as(ip_), len(sp),
                                                     out.ctypes.data_as(C.POINTER(C.c_float)))
        return rc, out

    def batch_segments(self, job: int) -> list:
        L = self.L
        out = []
        for i in range(L.whisper_mi355x_batch_n_segments(self.ptr, job)):
            toks = []
            for t in range(L.whisper_mi355x_batch_segment_n_tokens(self.ptr, job, i)):
                d = L.whisper_mi355x_batch_token_data(self.ptr, job, i, t)
                toks.append((d.id, d.tid, d.p, d.plog))
            out.append(Segment(L.whisper_mi355x_batch_segment_t0(self.ptr, job, i),
                               L.whisper_mi355x_batch_segment_t1(self.ptr, job, i),
                               L.whisper_mi355x_batch_segment_text(self.ptr, job, i), toks))
        return out

    def decisions(self, job: int = 0) -> list:
        """Per-window temperature-fallback decisions of the last full (job 0) / full_batch call."""
        cap = 256
        buf = (WindowDecision * cap)()
        n = self.L.whisper_mi355x_window_decisions(self.ptr, job, buf, cap)
        if n < 0:  # more windows than the buffer holds (> ~2 h of audio): retry with the returned count
            cap = -n
            buf = (WindowDecision * cap)()
            n = self.L.whisper_mi355x_window_decisions(self.ptr, job, buf, cap)
        assert n >= 0, n
        return [{f: getattr(d, f) for f, _ in WindowDecision._fields_ if f != "pad"} for d in buf[:n]]

    def info(self) -> dict:
        """whisper_mi355x_state_info: cross form of the last call, workspace slots, cross-cache slots,
        decode graphs kept, whether the state came from the context's pool."""
        out = (C.c_int * 5)()
        assert self.L.whisper_mi355x_state_info(self.ptr, out) == 5
        return dict(direct=bool(out[0]), cap_jobs=out[1], cap_cross=out[2], graphs=out[3], pooled=bool(out[4]))

    def pdec_give_ups(self) -> int:
        """Persistent decode launches of this state that gave up and were re-run on the per-kernel path."""
        return int(self.L.whisper_mi355x_pdec_give_ups(self.ptr))

    def phase_ms(self):
        out = (C.c_double * 5)()
        self.L.whisper_mi355x_phase_ms(self.ptr, out)
        return dict(zip(["mel", "encode", "prefill", "decode", "logits"], list(out)))

    def close(self):
        if self.ptr:
            self.L.whisper_free_state(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class WhisperEngine:
    """The C++ mirror of src-tauri/src/whisper.rs WhisperEngine (host/whisper_engine.cpp)."""

    NO_MODEL = -3

    def __init__(self):
        if not os.path.exists(ENGINE_LIB_PATH):
            raise RuntimeError(f"{ENGINE_LIB_PATH} missing: build with `make -C nobs-whisper_amd`")
        L = C.CDLL(ENGINE_LIB_PATH)
        L.nobs_engine_new.restype = C.c_void_p
        L.nobs_engine_free.argtypes = [C.c_void_p]
        L.nobs_engine_load.argtypes = [C.c_void_p, C.c_char_p]
        L.nobs_engine_is_loaded.argtypes = [C.c_void_p]
        L.nobs_engine_transcribe.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_int, C.c_char_p, C.c_char_p,
                                             C.c_char_p, C.c_char_p, C.c_int]
        L.nobs_engine_transcribe_chunked.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_int),
                                                     C.c_int, C.c_char_p, C.c_char_p, C.c_char_p, C.c_int]
        self.L = L
        self.ptr = L.nobs_engine_new()

    def load_model(self, path: str) -> int:
        return self.L.nobs_engine_load(self.ptr, path.encode())

    def is_loaded(self) -> bool:
        return bool(self.L.nobs_engine_is_loaded(self.ptr))

    def transcribe(self, audio, language=None, vocabulary=None, context=None):
        """Returns (rc, text): rc 0 ok, -1 LoadError, -2 TranscriptionError, -3 NoModel."""
        import numpy as np
        a = np.ascontiguousarray(audio, dtype=np.float32)
        buf = C.create_string_buffer(1 << 20)
        enc = lambda s: s.encode() if s is not None else None  # noqa: E731
        rc = self.L.nobs_engine_transcribe(self.ptr, a.ctypes.data_as(C.POINTER(C.c_float)), len(a), enc(language),
                                           enc(vocabulary), enc(context), buf, len(buf))
        return (0, buf.value.decode("utf-8", "replace")) if rc >= 0 else (rc, None)

    def transcribe_chunked(self, chunks, language=None, vocabulary=None):
        """whisper.rs:152-197: sequential transcribe calls, each prompted with the previous non-empty
        result; results joined with a space. Returns (rc, text)."""
        import numpy as np
        arrs = [np.ascontiguousarray(c, dtype=np.float32) for c in chunks]
        ptrs = (C.POINTER(C.c_float) * len(arrs))(*[a.ctypes.data_as(C.POINTER(C.c_float)) for a in arrs])
        lens = (C.c_int * len(arrs))(*[len(a) for a in arrs])
        buf = C.create_string_buffer(1 << 20)
        enc = lambda s: s.encode() if s is not None else None  # noqa: E731
        rc = self.L.nobs_engine_transcribe_chunked(self.ptr, ptrs, lens, len(arrs), enc(language), enc(vocabulary),
                                                   buf, len(buf))
        return (0, buf.value.decode("utf-8", "replace")) if rc >= 0 else (rc, None)

    def __del__(self):
        try:
            self.L.nobs_engine_free(self.ptr)
        except Exception:
            pass


def _engine_lib():
    return C.CDLL(ENGINE_LIB_PATH)


def _stream_lib():
    L = C.CDLL(ENGINE_LIB_PATH)
    fp = C.POINTER(C.c_float)
    L.nobs_audio_buffer_new.restype = C.c_void_p
    L.nobs_audio_buffer_new.argtypes = [C.c_uint]
    L.nobs_audio_buffer_free.argtypes = [C.c_void_p]
    L.nobs_audio_buffer_push.argtypes = [C.c_void_p, fp, C.c_long]
    L.nobs_audio_buffer_has_silence_boundary.argtypes = [C.c_void_p]
    L.nobs_audio_buffer_take.restype = C.c_long
    L.nobs_audio_buffer_take.argtypes = [C.c_void_p, C.c_int, fp, C.c_long]
    L.nobs_audio_buffer_info.argtypes = [C.c_void_p, C.POINTER(C.c_long), fp]
    L.nobs_calculate_rms.restype = C.c_float
    L.nobs_calculate_rms.argtypes = [fp, C.c_long]
    return L


def calculate_rms(x) -> float:
    """audio.rs:364-370 through the C++ mirror (host/audio_buffer.cpp)."""
    import numpy as np
    a = np.ascontiguousarray(x, dtype=np.float32)
    return float(_stream_lib().nobs_calculate_rms(a.ctypes.data_as(C.POINTER(C.c_float)), len(a)))


class AudioBuffer:
    """audio.rs:29-241 AudioBuffer through the C++ mirror (host/audio_buffer.cpp): same method names;
    take_* return a float32 array or None (Rust Option)."""

    def __init__(self, sample_rate: int = 48000):
        self.L = _stream_lib()
        self.ptr = self.L.nobs_audio_buffer_new(sample_rate)
        if not self.ptr:
            raise ValueError(f"unsupported sample rate {sample_rate}")

    @classmethod
    def with_sample_rate(cls, sample_rate: int):
        return cls(sample_rate)

    def push_samples(self, x):
        import numpy as np
        a = np.ascontiguousarray(x, dtype=np.float32)
        self.L.nobs_audio_buffer_push(self.ptr, a.ctypes.data_as(C.POINTER(C.c_float)), len(a))

    def _info(self):
        out, nf = (C.c_long * 4)(), C.c_float()
        self.L.nobs_audio_buffer_info(self.ptr, out, C.byref(nf))
        return list(out), nf.value

    def __len__(self):
        return self._info()[0][0]

    def is_empty(self) -> bool:
        return len(self) == 0

    @property
    def last_speech_pos(self) -> int:
        return self._info()[0][1]

    @property
    def overlap_len(self) -> int:
        return self._info()[0][2]

    @property
    def noise_floor_frames(self) -> int:
        return self._info()[0][3]

    def get_noise_floor(self) -> float:
        return self._info()[1]

    def has_silence_boundary(self) -> bool:
        return bool(self.L.nobs_audio_buffer_has_silence_boundary(self.ptr))

    def _take(self, kind):
        import numpy as np
        info = self._info()[0]
        out = np.zeros(info[0] + info[2] + 1, np.float32)
        n = self.L.nobs_audio_buffer_take(self.ptr, kind, out.ctypes.data_as(C.POINTER(C.c_float)), len(out))
        assert n >= 0, n
        return None if (n == 0 and kind != 2) else out[:n].copy()

    def take_chunk_at_silence(self):
        return self._take(0)

    def take_forced_chunk(self):
        return self._take(1)

    def take(self):
        return self._take(2)

    def __del__(self):
        try:
            self.L.nobs_audio_buffer_free(self.ptr)
        except Exception:
            pass


def build_initial_prompt(vocabulary, context):
    """whisper.rs:98-105 through the C++ mirror: None when the match falls through."""
    L = _engine_lib()
    L.nobs_build_initial_prompt.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int]
    buf = C.create_string_buffer(1 << 16)
    enc = lambda s: s.encode() if s is not None else None  # noqa: E731
    n = L.nobs_build_initial_prompt(enc(vocabulary), enc(context), buf, len(buf))
    return None if n == -1 else buf.value.decode()


def utf8_lossy(data: bytes) -> bytes:
    """The mirror's String::from_utf8_lossy (segment.to_str_lossy, whisper.rs:137)."""
    L = _engine_lib()
    L.nobs_utf8_lossy.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int]
    buf = C.create_string_buffer(3 * len(data) + 16)
    n = L.nobs_utf8_lossy(data, len(data), buf, len(buf))
    assert n >= 0
    return buf.raw[:n]


def filter_hallucinations(text: str) -> str:
    """whisper.rs:233-260 via the C++ mirror (no device needed)."""
    L = C.CDLL(ENGINE_LIB_PATH)
    L.nobs_filter_hallucinations.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
    buf = C.create_string_buffer(len(text.encode()) * 4 + 16)
    n = L.nobs_filter_hallucinations(text.encode(), buf, len(buf))
    assert n >= 0
    return buf.value.decode()


# ---- audio.rs mirror (src-tauri/src/audio.rs) over the GPU front-end ---------------------------------
WHISPER_SAMPLE_RATE = 16000   # audio.rs:7
CHUNK_OVERLAP_MS = 200        # audio.rs:15
MIN_CHUNK_DURATION_MS = 1000  # audio.rs:343


def _ptr_table(arrays):
    import numpy as np
    arrs = [np.ascontiguousarray(a, dtype=np.float32) for a in arrays]
    tab = (C.c_void_p * max(1, len(arrs)))(*[a.ctypes.data for a in arrs])
    n = (C.c_int * max(1, len(arrs)))(*[len(a) for a in arrs])
    return arrs, tab, n


def find_silence_boundaries_batch(clips, sample_rate: int, device: int = 0, with_rms: bool = False):
    """audio.rs:400-467 for every clip at once on the GPU: (boundaries per clip, noise floors, and
    with_rms the 20 ms window RMS rows)."""
    import numpy as np
    arrs, tab, n = _ptr_table(clips)
    nc = len(arrs)
    if nc == 0:
        return ([], [], []) if with_rms else ([], [])
    min_chunk = sample_rate * MIN_CHUNK_DURATION_MS // 1000
    cap = max(len(a) for a in arrs) // max(1, min_chunk) + 2
    counts = np.zeros(nc, np.int32)
    b = np.zeros((nc, cap), np.int32)
    nf = np.zeros(nc, np.float32)
    ws = sample_rate // 50
    stride = max(1, max(len(a) for a in arrs) // ws)
    rms = np.zeros((nc, stride), np.float32) if with_rms else None
    ip, fp = C.POINTER(C.c_int), C.POINTER(C.c_float)
    rc = lib().whisper_mi355x_find_silence_boundaries(
        device, tab, n, nc, sample_rate, False, counts.ctypes.data_as(ip), b.ctypes.data_as(ip), cap,
        nf.ctypes.data_as(fp), rms.ctypes.data_as(fp) if with_rms else None, stride)
    if rc != 0:
        raise RuntimeError(f"whisper_mi355x_find_silence_boundaries: {rc}")
    bounds = [b[c, :counts[c]].tolist() for c in range(nc)]
    if with_rms:
        return bounds, nf.tolist(), [rms[c, :len(arrs[c]) // ws].copy() for c in range(nc)]
    return bounds, nf.tolist()


def find_silence_boundaries(audio, sample_rate: int, device: int = 0) -> list:
    """audio.rs:400 find_silence_boundaries(audio, sample_rate) -> Vec<usize>."""
    return find_silence_boundaries_batch([audio], sample_rate, device)[0][0]


def split_at_silences_with_overlap(audio, boundaries, sample_rate: int) -> list:
    """audio.rs:474-507: chunks audio[max(start - overlap, 0) : boundary], overlap 200 ms."""
    if not boundaries:
        return [audio[:]]
    overlap = sample_rate * CHUNK_OVERLAP_MS // 1000
    chunks, start = [], 0
    for b in boundaries:
        if start < b < len(audio):
            chunks.append(audio[max(start - overlap, 0):b])
            start = b
    if start < len(audio):
        chunks.append(audio[max(start - overlap, 0):])
    return chunks


def split_at_silences(audio, boundaries) -> list:
    """audio.rs:469-471."""
    return split_at_silences_with_overlap(audio, boundaries, WHISPER_SAMPLE_RATE)


def resample_batch(clips, input_sample_rate: int, device: int = 0) -> list:
    """audio.rs:331-337 resample_chunk for every clip at once on the GPU."""
    import numpy as np
    arrs, tab, n = _ptr_table(clips)
    if not arrs:
        return []
    L = lib()
    outs = [np.zeros(max(1, L.whisper_mi355x_resample_len(len(a), input_sample_rate)), np.float32) for a in arrs]
    otab = (C.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
    rc = L.whisper_mi355x_resample_chunk(device, tab, n, len(arrs), input_sample_rate, False, otab)
    if rc != 0:
        raise RuntimeError(f"whisper_mi355x_resample_chunk: {rc}")
    return [o[:L.whisper_mi355x_resample_len(len(a), input_sample_rate)] for o, a in zip(outs, arrs)]


def resample_chunk(audio, input_sample_rate: int, device: int = 0):
    """audio.rs:331 resample_chunk(audio, input_sample_rate) -> Vec<f32> at 16 kHz."""
    return resample_batch([audio], input_sample_rate, device)[0]
