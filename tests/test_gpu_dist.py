"""The engine's multi-rank piece on one GPU: a context created with load_weights = false (a rank
that receives its weights over RCCL, bench.py / SURVEY.md §8e) parses the file for sizes only and
lays out an arena byte-identical in size to the loading rank's. Filling it with the loading rank's
arena (the ncclBroadcast payload; a device copy stands in for RCCL, which needs one GPU per rank)
must give the same transcription, bit for bit. RCCL itself (whisper_mi355x_broadcast_weights) is a
no-op at world size 1 and is exercised by the driver's multi-GPU bench."""
import ctypes as C

import pytest

from make_model import synthetic_pcm

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", ["F16", "BF16"])
def test_sizes_only_context_after_arena_copy(wrs, tiny_model, dtype):
    L = wrs.lib()
    dt = getattr(wrs, dtype)
    a = wrs.WhisperContext(tiny_model, dtype=dt)
    b = wrs.WhisperContext(tiny_model, dtype=dt, load_weights=False)
    pa, na = C.c_void_p(), C.c_size_t()
    pb, nb = C.c_void_p(), C.c_size_t()
    assert L.whisper_mi355x_weight_arena(a.ptr, C.byref(pa), C.byref(na)) == 0
    assert L.whisper_mi355x_weight_arena(b.ptr, C.byref(pb), C.byref(nb)) == 0
    assert na.value == nb.value and na.value > 0
    assert L.whisper_mi355x_memcpy(b.ptr, pb, pa, na.value, 3) == 0  # hipMemcpyDeviceToDevice
    assert L.whisper_mi355x_broadcast_weights(b.ptr, b"\0" * 128, 0, 1) == 0  # world 1: no-op
    p = wrs.reference_full_params("en")
    p.temperature_inc = 0.0
    pcm = synthetic_pcm(2)
    out = []
    for ctx in (a, b):
        st = ctx.create_state()
        assert st.full(p, pcm) == 0
        out.append([([t[0] for t in s.tokens], s.t0, s.t1, s.text) for s in st.segments()])
        st.close()
    assert out[0] == out[1] and len(out[0]) > 0
    a.close()
    b.close()
