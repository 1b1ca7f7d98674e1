"""North-star logits bound: "greedy-decode token IDs match ... bit-exact (logits within 1e-3 fp16)".

Metric: per decode step, max_v |logit_gpu[v] - logit_oracle[v]| / max_v |logit_oracle[v]|,
on the f16 path (the GGML file's own weight type, whisper.cpp's numerics), teacher-forced along the
oracle's own greedy sequence so that both sides see the same prefix at every step. Bar: <= 1e-3 at
every step, on tiny.en, base, small and large-v3 shapes ("+conf" decoders, whose logit range is that
of a trained model: max |logit| ~ 20-40).
"""
import ctypes as C

import numpy as np
import pytest

from make_model import synthetic_pcm
from oracle_py import Oracle, reference_params

pytestmark = pytest.mark.gpu

REL_TOL = 1e-3


@pytest.mark.parametrize("shape", ["tiny.en+conf", "base+conf", "small-4L+conf", "large-v3-2L+conf"])
def test_f16_teacher_forced_logits_rel_1e3(wrs, shape):
    from conftest import model_path
    path = model_path(shape)
    pcm = synthetic_pcm(0)
    o = Oracle(path, mode=1, n_threads=16)
    rp = reference_params("en")
    rp.temperature_inc = 0.0
    ref = o.full(pcm, rp)
    seq = [t for s in ref["segments"] for t in s["tokens"]][:32]
    L = wrs.lib()
    ctx = wrs.WhisperContext(path, dtype=wrs.F16)
    st = ctx.create_state()
    assert L.whisper_pcm_to_mel_with_state(ctx.ptr, st.ptr, pcm.ctypes.data_as(C.POINTER(C.c_float)), len(pcm), 1) == 0
    assert L.whisper_encode_with_state(ctx.ptr, st.ptr, 0, 1) == 0
    sot = L.whisper_token_sot(ctx.ptr)
    prompt = [sot]
    if L.whisper_is_multilingual(ctx.ptr):
        prompt += [sot + 1, L.whisper_token_transcribe(ctx.ptr)]
    V = L.whisper_n_vocab(ctx.ptr)
    toks = prompt + seq
    o.mel(pcm)
    o.encode(0)
    o.kv_clear()
    rel, absd, scale = [], [], []
    for i in range(len(prompt) - 1, len(toks)):
        chunk = toks[:len(prompt)] if i == len(prompt) - 1 else [toks[i]]
        n_past = 0 if i == len(prompt) - 1 else i
        arr = (C.c_int * len(chunk))(*chunk)
        assert L.whisper_decode_with_state(ctx.ptr, st.ptr, arr, len(chunk), n_past, 1) == 0
        g = np.ctypeslib.as_array(L.whisper_get_logits_from_state(st.ptr), shape=(len(chunk) * V,))[-V:].copy()
        r = o.decode(chunk, n_past)[-1]
        d = float(np.abs(g.astype(np.float64) - r).max())
        m = float(np.abs(r).max())
        rel.append(d / m)
        absd.append(d)
        scale.append(m)
        assert int(np.argmax(g)) == int(np.argmax(r)) or np.sort(r)[-1] - np.sort(r)[-2] < 2 * d, i
    st.close()
    ctx.close()
    o.close()
    k = int(np.argmax(rel))
    print(f"{shape}: {len(rel)} steps, max rel {max(rel):.2e} (|d| {absd[k]:.4f} of max|logit| {scale[k]:.2f}), "
          f"median rel {np.median(rel):.2e}")
    assert max(rel) <= REL_TOL, (shape, max(rel), absd[k], scale[k])
