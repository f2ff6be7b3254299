"""bench.py's N > 1 orchestration, driven on CPU: world-size-2 (and 4) ``gloo`` process
groups run ``bench.run`` with the CPU oracle injected as the attention (test
infrastructure; on the GPU box the same code calls the HIP forward over RCCL). Checks
the strong / weak shard plans, that the all-gathered output of the sharded run equals
the global attention, and the JSON contract fields of the line rank 0 prints."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_plan_strong_and_weak():
    for world in (1, 2, 4, 8):
        spans = [bench.shard_plan((8, 16, 4096, 64), world, r) for r in range(world)]
        assert spans[0]["bh_lo"] == 0 and spans[-1]["bh_hi"] == 128
        assert all(a["bh_hi"] == b["bh_lo"] for a, b in zip(spans, spans[1:]))
        assert all(s["global_shape"] == (8, 16, 4096, 64) for s in spans)
        assert spans[0]["shard_shape"] == (8 // world, 16, 4096, 64)
        c4 = bench.shard_plan((64, 16, 16384, 128), world, world - 1)
        assert c4["shard_shape"] == (64 // world, 16, 16384, 128)
        assert c4["bh_hi"] == 1024
        w = bench.shard_plan((8, 16, 4096, 64), world, world - 1, "weak")
        assert w["shard_shape"] == (8, 16, 4096, 64) and w["global_shape"] == (8 * world, 16, 4096, 64)
    # more ranks than batch rows: one contiguous (1, BH/W) block per rank
    p = bench.shard_plan((2, 8, 64, 16), 4, 3)
    assert p["shard_shape"] == (1, 4, 64, 16) and (p["bh_lo"], p["bh_hi"]) == (12, 16)
    with pytest.raises(ValueError):
        bench.shard_plan((1, 3, 64, 16), 2, 0)


def test_make_shard_is_slice_of_global():
    g = bench.make_shard(torch, (2, 4, 8, 4), 0, torch.float32, 1, "cpu")
    s = bench.make_shard(torch, (1, 4, 8, 4), 4, torch.float32, 1, "cpu")
    assert torch.equal(g[1], s[0])


def _oracle_attn(q, k, v, causal, out):
    from oracle import attention as A
    o, _, _ = A.attention_fwd(q.float().numpy(), k.float().numpy(), v.float().numpy(), causal)
    out.copy_(torch.from_numpy(o))


def _worker(rank, world, port, argv, q_out, bf16_in=False):
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        args = bench.parse_args(argv)
        # bf16_in: the headline's types (bf16 Q/K/V, fp32 O); else fp32 throughout
        res, gathered, _ = bench.run(args, _oracle_attn, torch, dist, world, rank, "cpu",
                                     torch.bfloat16 if bf16_in else torch.float32,
                                     esize=2 if bf16_in else 4, out_esize=4)
        q_out.put((rank, res, gathered.float().numpy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface the failure in the parent
        import traceback
        q_out.put((rank, "error", traceback.format_exc() + repr(e)))


def _run_world(world, argv, bf16_in=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, argv, q, bf16_in)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, res, arr = q.get(timeout=240)
        assert res != "error", arr
        out[rank] = (res, arr)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("world,split", [(2, "strong"), (2, "weak"), (4, "strong")])
@pytest.mark.parametrize("causal", [False, True])
def test_bench_multi_rank_cpu(world, split, causal):
    shape = (2, 4, 48, 16)
    argv = ["--gpus", str(world), "--steps", "2", "--warmup", "1", "--split", split,
            "--chunks", "2", "--shape", *map(str, shape)] + (["--causal"] if causal else [])
    out = _run_world(world, argv)
    res, gathered = out[0]
    # the JSON contract fields
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline", "end_to_end"):
        assert key in res, key
    assert res["n_gpus"] == world and res["scaling"] == split and res["steps"] == 2
    assert res["value"] > 0 and res["end_to_end"]["tflops"] > 0
    # B*H divides world * 2: the end-to-end leg is the overlapped chunked gather (whose
    # gathered output is checked below), with the serial gather reported beside it
    assert res["end_to_end"]["chunks"] == 2 and res["end_to_end_serial"]["tflops"] > 0
    glob = (shape[0] * world,) + shape[1:] if split == "weak" else shape
    assert tuple(res["config"][k] for k in ("B", "H", "N", "d")) == glob
    # the gathered shards are the global attention, in global head order
    from oracle import attention as A
    q, k, v = (bench.make_shard(torch, glob, 0, torch.float32, s, "cpu").numpy() for s in (1, 2, 3))
    o_ref, _, _ = A.attention_fwd(q, k, v, causal)
    got = gathered.reshape(o_ref.shape)
    np.testing.assert_allclose(got, o_ref, atol=1e-6)
    # every rank holds the same gathered tensor
    for r in range(1, world):
        np.testing.assert_array_equal(out[r][1], gathered)


def test_gpus_must_match_world():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, env={**os.environ, "WORLD_SIZE": "1"})
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_occupancy_chunks_rule():
    """The end-to-end leg's default chunk count (minitorch/shard.py occupancy_chunks) for
    BASELINE configs 3 and 4 at 1, 2, 4 and 8 ranks: a chunk keeps at least one workgroup per
    CU of the forward's default (8-wave, non-split) form."""
    from minitorch.shard import occupancy_chunks, forward_workgroups_per_head
    c3, c4 = (8, 16, 4096, 64), (64, 16, 16384, 128)
    assert [occupancy_chunks(*c3, w) for w in (1, 2, 4, 8)] == [4, 2, 1, 1]
    assert [occupancy_chunks(*c4, w) for w in (1, 2, 4, 8)] == [4, 4, 4, 4]
    for shape in (c3, c4):
        for w in (1, 2, 4, 8):
            c = occupancy_chunks(*shape, w)
            rows = shape[0] * shape[1] // w
            assert rows % c == 0
            assert c == 1 or (rows // c) * forward_workgroups_per_head(shape[2], shape[3]) >= 256
    assert occupancy_chunks(8, 16, 4096, 64, 3) == 1   # B*H not divisible by the world


def test_bench_default_chunking_world4_bitwise():
    """gloo world 4: bench.run with the chunk count the rule picks (on a model chip of 2 CUs
    for this small shape) all-gathers an O bit-identical to the unchunked run's."""
    from minitorch.shard import occupancy_chunks
    shape = (4, 4, 48, 16)
    chosen = occupancy_chunks(*shape, 4, cus=2)
    assert chosen == 2
    base = ["--gpus", "4", "--steps", "1", "--warmup", "1", "--shape", *map(str, shape)]
    chunked = _run_world(4, base + ["--chunks", str(chosen)])
    serial = _run_world(4, base + ["--chunks", "1"])
    assert chunked[0][0]["end_to_end"]["chunks"] == chosen
    for r in range(4):
        np.testing.assert_array_equal(chunked[r][1], serial[r][1])


def test_bench_world8_chunked_and_unchunked_bitwise():
    """gloo world 8, the rank count of the driver's scaling run: bench.run on a scaled-down
    config 4 (d = 128 -> 32, N 16384 -> 64) with the 4 chunks occupancy_chunks picks for it on
    a model chip of 2 CUs (the C4 case: every rank's rows in 4 block-cyclic pieces), and
    unchunked (the C3 case at 8 ranks); both all-gather an O bit-identical to world 1's, and
    rank 0's line carries the end-to-end leg."""
    from minitorch.shard import occupancy_chunks
    shape = (16, 4, 64, 32)
    chosen = occupancy_chunks(*shape, 8, cus=2)
    assert chosen == 4
    base = ["--steps", "1", "--warmup", "1", "--shape", *map(str, shape)]
    one = _run_world(1, ["--gpus", "1"] + base)
    ref = one[0][1].reshape((-1,) + shape[2:])
    for chunks in (chosen, 1):
        out = _run_world(8, ["--gpus", "8"] + base + ["--chunks", str(chunks)])
        res = out[0][0]
        assert res["n_gpus"] == 8 and res["end_to_end"]["tflops"] > 0
        if chunks > 1:
            assert res["end_to_end"]["chunks"] == chunks
        for r in range(8):
            np.testing.assert_array_equal(out[r][1].reshape(ref.shape), ref)


def test_bench_bf16_in_fp32_out_chunked_world2():
    """The headline's types through the N > 1 legs: bf16 Q/K/V shards, fp32 O, the overlapped
    chunked all-gather (its pieces' O must be fp32 like the gathered tensor) and the serial one;
    the gathered output equals world 1's bitwise."""
    shape = (2, 4, 48, 16)
    argv = ["--gpus", "2", "--steps", "2", "--warmup", "1", "--chunks", "2", "--shape", *map(str, shape)]
    out2 = _run_world(2, argv, bf16_in=True)
    res, gathered = out2[0]
    assert res["end_to_end"]["chunks"] == 2 and res["config"]["output"] == "fp32 O"
    assert res["roofline"]["algorithmic_bytes"] == bench.fwd_bytes(1, 4, 48, 16, 2, 4)
    out1 = _run_world(1, ["--gpus", "1", "--steps", "2", "--warmup", "1", "--shape", *map(str, shape)], bf16_in=True)
    np.testing.assert_array_equal(gathered.reshape(-1), out1[0][1].reshape(-1))
