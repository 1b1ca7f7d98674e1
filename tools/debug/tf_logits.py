"""Teacher-forced F16 logits of the engine vs the oracle along the oracle's greedy sequence, plus the
encoder output error: python tools/debug/tf_logits.py SHAPE [clip] [dtype]"""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path
from make_model import synthetic_pcm
from oracle_py import Oracle, reference_params
wrs = load_whisper_rs()
shape = sys.argv[1]
clip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
dt = getattr(wrs, sys.argv[3]) if len(sys.argv) > 3 else wrs.F16
path = model_path(shape)
pcm = synthetic_pcm(clip)
o = Oracle(path, mode=1, n_threads=16)
rp = reference_params("en"); rp.temperature_inc = 0.0
ref = o.full(pcm, rp)
seq = [t for s in ref["segments"] for t in s["tokens"]][:40]
L = wrs.lib()
ctx = wrs.WhisperContext(path, dtype=dt)
st = ctx.create_state()
assert L.whisper_pcm_to_mel_with_state(ctx.ptr, st.ptr, pcm.ctypes.data_as(C.POINTER(C.c_float)), len(pcm), 1) == 0
assert L.whisper_encode_with_state(ctx.ptr, st.ptr, 0, 1) == 0
d = L.whisper_model_n_audio_state(ctx.ptr)
eo = np.empty((1500, d), np.float32)
L.whisper_mi355x_get_encoder_out(st.ptr, eo.ctypes.data_as(C.POINTER(C.c_float)), eo.size)
o.new_state(); o.mel(pcm); er = o.encode(0); o.kv_clear()
print(shape, "encoder max/mean abs err", float(np.abs(eo - er).max()), float(np.abs(eo - er).mean()))
sot = L.whisper_token_sot(ctx.ptr)
prompt = [sot, sot + 1, L.whisper_token_transcribe(ctx.ptr)] if L.whisper_is_multilingual(ctx.ptr) else [sot]
V = L.whisper_n_vocab(ctx.ptr)
toks = prompt + seq
worst = 0.0
for i in range(len(prompt) - 1, len(toks)):
    chunk = toks[:len(prompt)] if i == len(prompt) - 1 else [toks[i]]
    n_past = 0 if i == len(prompt) - 1 else i
    arr = (C.c_int * len(chunk))(*chunk)
    assert L.whisper_decode_with_state(ctx.ptr, st.ptr, arr, len(chunk), n_past, 1) == 0
    g = np.ctypeslib.as_array(L.whisper_get_logits_from_state(st.ptr), shape=(len(chunk) * V,))[-V:].copy()
    r = o.decode(chunk, n_past)[-1]
    e = float(np.abs(g - r).max()); worst = max(worst, e)
    top2 = np.sort(r)[-2:]
    print(i, "max|dlogit| %.4f" % e, "argmax", int(np.argmax(g)), int(np.argmax(r)), "gap %.3f" % (top2[1] - top2[0]))
print("worst", worst)
