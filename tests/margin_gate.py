"""The close-call margin gate for reduced-precision runs (bf16, fp8) against the f16-numerics oracle.

A greedy decode of lower precision may flip a choice the oracle made by a small margin, never a
confident one. For every token the oracle kept in its segments this module gives the smallest
margin (top-2 log-probability gap, or the gap of the "sum p(timestamps) > max p(text)" rule) over
the oracle's decode steps since the previous kept token of the same window, up to and including
its own; a flip on a dropped step (a segment-opening timestamp) surfaces at the next kept token.

Multi-window runs (> 30 s, or a window that ends early): the oracle records the window (seek) of
every step and of every segment, so each window's kept tokens are aligned with that window's own
steps. Comparison stops at the first difference: later windows depend on the earlier ones' seek
and prompt carry-over. Use with temperature_inc = 0 (one greedy attempt per window).
"""


def kept_token_margins(ref):
    """(tokens, margins) of the oracle result `ref` (oracle_py.Oracle.full), flattened over windows."""
    seeks = ref["step_seeks"]
    toks = ref["step_tokens"]
    marg = [float(x) for x in ref["margins"]]
    assert len(seeks) == len(toks) == len(marg), (len(seeks), len(toks), len(marg))
    by_seek = {}
    for i, s in enumerate(seeks):
        by_seek.setdefault(s, []).append(i)
    out_t, out_m = [], []
    pos = {}
    for seg in ref["segments"]:
        steps = by_seek[seg["seek"]]
        i = pos.get(seg["seek"], 0)
        for t in seg["tokens"]:
            j = i
            while toks[steps[j]] != t:
                j += 1
            out_t.append(t)
            out_m.append(min(marg[steps[k]] for k in range(i, j + 1)))
            i = j + 1
        pos[seg["seek"]] = i
    return out_t, out_m


def assert_diverges_only_at_close_calls(got, exp, margins, gap, min_confident=0, min_prefix=None):
    """got == exp up to the first difference, which must fall on a token the oracle decided by at
    most `gap` nats; and the identical prefix holds at least min(min_confident, C) tokens that the
    oracle decided by MORE than `gap` (C = how many such tokens exp has), or is at least `min_prefix`
    tokens long (default 2 * min_confident), so that a case whose first steps are all close calls
    cannot pass having checked nothing. (A small-4L bf16 clip kept 12 identical tokens, 3 of them
    confident, and flipped a 0.1-nat call at token 12: evidence, not a vacuous pass.) Returns the
    prefix length."""
    if min_prefix is None:
        min_prefix = 2 * min_confident
    n = 0
    while n < len(exp) and n < len(got) and got[n] == exp[n]:
        n += 1
    if n < len(exp) and n < len(got):
        assert n < len(margins) and margins[n] <= gap, \
            f"diverged at token {n} where the oracle's margin is {margins[n]:.3f} nats (> {gap})"
    elif n < len(exp):
        # the run ended (EOT, window end) where the oracle went on with token n: a flip of that step
        assert margins[n] <= gap, f"ended at token {n} where the oracle's margin is {margins[n]:.3f} nats (> {gap})"
    confident = sum(1 for m in margins[:len(exp)] if m > gap)
    covered = sum(1 for m in margins[:n] if m > gap)
    assert covered >= min(min_confident, confident) or n >= min(min_prefix, len(exp)), \
        f"identical prefix {n} (< {min_prefix}) holds {covered} confident tokens < {min(min_confident, confident)}"
    return n


DEC_KEYS = ("seek", "temp_idx", "failed0", "logprob_fail0", "result_len0", "no_speech")


def assert_closed_before_divergence(segs, decs, ref, n):
    """Near-tie runs (VERDICT r4 "next" #1): besides the identical token prefix of length n (kept tokens,
    as assert_diverges_only_at_close_calls returns it), everything that was decided before the divergence
    must equal the oracle's:
      * every segment that closes before it (at least one identical kept token follows the segment):
        its tokens, t0, t1 and text;
      * every window that ends before the window of the first differing token: its per-window
        decisions (seek, temperature index, greedy failure, logprob failure, result length, no-speech).
    segs: GPU segments (whisper_rs.Segment), decs: GPU decisions (dicts), ref: oracle_py Oracle.full.
    When the whole token sequence is identical (a near tie that did not flip), everything is compared.
    Returns (segments compared, windows compared)."""
    rsegs = ref["segments"]
    n_kept = sum(len(s["tokens"]) for s in rsegs)
    got_tokens = [t[0] for s in segs for t in s.tokens]
    if n == n_kept and len(got_tokens) == n_kept:
        n_seg, div_seek = len(rsegs), None
    else:
        n_seg, cum = 0, 0
        for s in rsegs:
            cum += len(s["tokens"])
            if cum >= n:
                break
            n_seg += 1
        # the window of the first differing kept token (or, when the GPU only went on past the oracle's
        # last token, the window of that last token)
        k, cum, div_seek = min(n, n_kept - 1), 0, rsegs[-1]["seek"] if rsegs else 0
        for s in rsegs:
            if k < cum + len(s["tokens"]):
                div_seek = s["seek"]
                break
            cum += len(s["tokens"])
    assert len(segs) >= n_seg, (len(segs), n_seg)
    for i in range(n_seg):
        g, r = segs[i], rsegs[i]
        assert ([t[0] for t in g.tokens], g.t0, g.t1) == (r["tokens"], r["t0"], r["t1"]), (i, g.t0, g.t1, r["t0"], r["t1"])
        assert g.text == r["text"], (i, g.text, r["text"])
    rdec = ref["decisions"] if div_seek is None else [d for d in ref["decisions"] if d["seek"] < div_seek]
    assert len(decs) >= len(rdec), (len(decs), len(rdec))
    for k, d in enumerate(rdec):
        assert tuple(decs[k][x] for x in DEC_KEYS) == tuple(d[x] for x in DEC_KEYS), (k, decs[k], d)
    return n_seg, len(rdec)
