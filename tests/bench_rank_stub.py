"""Per-rank entry of the CPU rehearsal of ``bench.py --gpus N`` (tests/test_bench_dp.py): started by
bench.launch_ranks through torch.distributed.run exactly as the 8-GPU launch starts bench.py, it parses
bench's own arguments, sets up the rank with bench.setup_ranks (gloo on the CPU under
SD_AMD_BENCH_REHEARSAL=cpu) and runs bench's data-parallel step code (rank_inputs -> make_one_step ->
timed_steps -> all-gather -> dp_report) with CPU stand-ins for the GPU sampler and decoder.  Rank 0 writes the
gathered batch and every rank's (RANK, LOCAL_RANK, WORLD_SIZE) to $BENCH_STUB_OUT; rank
$BENCH_STUB_FAIL_RANK (if set) exits with status 7 before the step, to check that a failing rank's
status reaches the launcher's caller.  Not a test module (no test_ prefix)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import bench
    from test_bench_dp import _StubLD, _StubSampler
    args = bench.make_parser().parse_args()
    world, rank, local, dist, device = bench.setup_ranks(args)
    if os.environ.get("BENCH_STUB_FAIL_RANK") == str(rank):
        sys.exit(7)
    import torch.distributed as tdist
    B, L = args.batch or 3, 8
    xT, ctx = bench.rank_inputs(2024, world, rank, B, (4, L, L), (5, 16), device)
    gathered = torch.empty(world * B, 3, 8 * L, 8 * L, dtype=torch.float16) if dist else None
    gt = bench.GatherTimer(device)
    one_step = bench.make_one_step(_StubSampler(), _StubLD(), xT, ctx, args.ddim_steps, world, gathered, gt)
    img, elapsed = bench.timed_steps(one_step, args.steps, args.warmup, bench.make_barrier(dist, device), device, gt)
    n_timed = len(gt.marks)
    dp = bench.dp_report(img, gathered, rank, world, device, gt)
    plumb = torch.tensor([rank, local, world, int(os.environ["RANK"]), int(os.environ["LOCAL_RANK"])],
                         dtype=torch.int64)
    allp = [torch.empty_like(plumb) for _ in range(world)]
    tdist.all_gather(allp, plumb)
    if rank == 0:
        torch.save({"gathered": gathered, "plumbing": torch.stack(allp), "elapsed": elapsed, "dp": dp,
                    "n_timed_gathers": n_timed}, os.environ["BENCH_STUB_OUT"])
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
