"""bench.py's data-parallel structure on the CPU (gloo, world_size 2) and its launcher checks.

The per-rank step is bench's own code — ``rank_inputs`` (shard of the host-generated global
batch), ``make_one_step`` (sample → decode → all-gather into the rank-major buffer) and
``timed_steps`` (warm-up, barrier-bracketed timed steps, max over ranks) — with the GPU sampler
and decoder replaced by CPU stand-ins built on the oracle's DDIM update.  ``sdd.gather`` is the
same ``all_gather_into_tensor`` call the nccl (RCCL) branch makes, so the gathered layout is the
one the 8-GPU run produces; it must equal the single-process result bit for bit.
Reference basis: samples of a batch never interact (``ldm/diffusion/ddim.py:114-165``)."""
import os
import socket
import subprocess
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _StubSampler:
    """DDIMSampler.sample's signature; ε = a per-row function of (x, context) → shard-independent."""

    def sample(self, S, batch_size, shape, conditioning=None, eta=0.0, x_T=None, verbose=False, log_every_t=100):
        from oracle import schedule as osch
        tab = osch.ddim_tables(S, 0.0)
        x = x_T.float().clone()
        assert x.shape == (batch_size,) + tuple(shape)
        bias = conditioning.float().mean(dim=(1, 2)).view(-1, 1, 1, 1)
        for i in range(S):
            index = S - i - 1
            eps = torch.tanh(x) * 0.5 + bias
            xp, _ = osch.ddim_step(x.numpy(), eps.numpy(), osch.ddim_step_scalars(tab, index))
            x = torch.from_numpy(xp)
        return x, {}


class _StubLD:
    def decode_first_stage(self, z):
        return torch.nn.functional.interpolate(z[:, :3], scale_factor=8, mode="nearest")


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cpu")
        B, L = 3, 8
        xT, ctx = bench.rank_inputs(2024, world, rank, B, (4, L, L), (5, 16), dev)
        assert xT.shape == (B, 4, L, L) and ctx.shape == (B, 5, 16)
        gathered = torch.empty(world * B, 3, 8 * L, 8 * L, dtype=torch.float16)
        gt = bench.GatherTimer(dev)
        one_step = bench.make_one_step(_StubSampler(), _StubLD(), xT, ctx, 4, world, gathered, gt)
        barrier = bench.make_barrier(True, dev)
        img, elapsed = bench.timed_steps(one_step, 2, 1, barrier, dev, gt)
        assert img.shape == (B, 3, 8 * L, 8 * L) and elapsed > 0
        assert len(gt.marks) == 2          # the timed steps' gathers only (warm-up dropped)
        dp = bench.dp_report(img, gathered, rank, world, dev, gt)
        # a corrupted slice (rank 1's image in the gathered buffer) is caught on every rank
        bad = gathered.clone()
        bad[B + 1, 0, 0, 0] += 1
        dp_bad = bench.dp_report(img, bad, rank, world, dev, gt)
        from sd_amd import distributed as sdd
        t = sdd.max_over_ranks(0.5 + rank)
        if rank == 0:
            out_q.put((gathered, t, dp, dp_bad))
    finally:
        dist.destroy_process_group()


def test_bench_dp_step_matches_single_process():
    import sd_amd_loader
    sd_amd_loader.load()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, t, dp, dp_bad = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import bench
    xg, cg = bench.rank_inputs(2024, 1, 0, world * 3, (4, 8, 8), (5, 16), torch.device("cpu"))
    z, _ = _StubSampler().sample(4, world * 3, (4, 8, 8), conditioning=cg, x_T=xg)
    ref = _StubLD().decode_first_stage(z).half()
    assert torch.equal(gathered, ref)
    assert t == 1.5
    # the self-verifying fields of the N > 1 bench line
    assert dp["ranks_seen"] == 2 and dp["backend"] == "gloo"
    assert dp["allgather_ms"] is not None and dp["allgather_ms"] >= 0
    assert dp["allgather_bytes_per_rank"] == 3 * 3 * 64 * 64 * 2
    assert dp["gather_slices_bitwise_equal"] is True and dp["gather_mismatched_ranks"] == 0
    assert dp_bad["gather_slices_bitwise_equal"] is False and dp_bad["gather_mismatched_ranks"] == 1


def _run_bench(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=env, timeout=300, cwd=ROOT)


def test_bench_refuses_more_gpus_than_visible():
    """--gpus N without a launcher spawns N ranks only if N GPUs are visible; otherwise it fails
    fast, non-zero, and never prints a bench line (here: no GPU at all)."""
    r = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"HIP_VISIBLE_DEVICES": ""})
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr
    assert '"metric"' not in r.stdout


def test_bench_rejects_world_size_mismatch():
    r = _run_bench(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr
    assert '"metric"' not in r.stdout


def _launch(n, tmp_path, extra_env=None):
    """bench.launch_ranks(n) as bench.py --gpus n runs it (GPU-free parent -> torch.distributed.run child
    -> one process per rank), with tests/bench_rank_stub.py as the rank entry, in a subprocess (the
    launcher ends with sys.exit(child status))."""
    out = str(tmp_path / "stub.pt")
    code = ("import sys, torch; sys.path.insert(0, %r); import bench; "
            "sys.argv = ['bench.py', '--gpus', '%d', '--steps', '2', '--warmup', '1', '--ddim-steps', '4']; "
            "torch.cuda.device_count = lambda: %d; "
            "bench.launch_ranks(%d, entry=%r)") % (ROOT, n, n, n, os.path.join(ROOT, "tests", "bench_rank_stub.py"))
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(SD_AMD_BENCH_REHEARSAL="cpu", BENCH_STUB_OUT=out, OMP_NUM_THREADS="1", **(extra_env or {}))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)
    return r, out


def test_launch_ranks_spawns_ranks_and_gathers_rank_major(tmp_path):
    """bench.launch_ranks(2) on the CPU: two ranks with RANK / LOCAL_RANK / WORLD_SIZE = (r, r, 2) from
    torch.distributed.run, bench.setup_ranks agreeing with them, and the all-gathered batch in rank-major
    order equal to the single-process result bit for bit."""
    r, out = _launch(2, tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    res = torch.load(out, weights_only=True)
    plumb = res["plumbing"].tolist()
    assert plumb == [[0, 0, 2, 0, 0], [1, 1, 2, 1, 1]]
    import bench
    xg, cg = bench.rank_inputs(2024, 1, 0, 2 * 3, (4, 8, 8), (5, 16), torch.device("cpu"))
    z, _ = _StubSampler().sample(4, 2 * 3, (4, 8, 8), conditioning=cg, x_T=xg)
    assert torch.equal(res["gathered"], _StubLD().decode_first_stage(z).half())
    assert res["elapsed"] > 0
    dp = res["dp"]
    assert dp["ranks_seen"] == 2 and dp["backend"] == "gloo" and dp["gather_slices_bitwise_equal"] is True
    assert dp["allgather_ms"] is not None and res["n_timed_gathers"] == 2


def test_launch_ranks_propagates_a_failing_rank(tmp_path):
    """A rank that dies (status 7) fails the whole launch: the launcher's caller exits non-zero and no
    bench line is printed."""
    r, _ = _launch(2, tmp_path, {"BENCH_STUB_FAIL_RANK": "1"})
    assert r.returncode != 0
    assert '"metric"' not in r.stdout
