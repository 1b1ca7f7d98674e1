"""Multi-rank path on the CPU (gloo, world_size 2): bench.py's chunk sharding and max-over-ranks
timing, and that transcribing each rank's shard independently gives exactly the single-process
result for every chunk (weak scaling with no data-path collective). The
per-chunk transcription here is the CPU oracle (test infrastructure), standing in for the GPU
engine which these CPU tests cannot run."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

BATCH = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _transcribe(model, cid):
    from make_model import synthetic_pcm
    from oracle_py import Oracle, reference_params
    o = Oracle(model, mode=1, n_threads=2)
    r = o.full(synthetic_pcm(cid, seconds=5), reference_params("en", fixed_tokens=6))
    o.close()
    assert r["rc"] == 0
    return [(s["t0"], s["t1"], s["text"], list(s["tokens"])) for s in r["segments"]]


def _worker(rank, world, port, model, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests"), os.path.join(root, "tools")]
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = bench.rank_chunk_ids(rank, BATCH)
    res = {cid: _transcribe(model, cid) for cid in ids}
    gathered = [None] * world
    dist.all_gather_object(gathered, res)
    t = bench.max_over_ranks(float(rank + 1) * 0.5, dist, "cpu")
    if rank == 0:
        q.put((gathered, t))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_matches_single_process(micro_model):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, micro_model, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, t = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 1.0  # max over ranks of 0.5, 1.0
    merged = {}
    for part in gathered:
        assert not (set(part) & set(merged)), "ranks transcribed overlapping chunks"
        merged.update(part)
    assert sorted(merged) == list(range(2 * BATCH))
    for cid, r in merged.items():
        assert r == _transcribe(micro_model, cid), f"chunk {cid}"
