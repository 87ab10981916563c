"""bench.py's own process, timed window repeated: is the first 20-step window after start-up slower than the
following ones (a one-time cost), or are all of them slower than 20-step windows inside a long run?
bench.timed_region is wrapped: after the real (first) window, WINDOWS more windows of the same K steps are timed,
half of them right after the previous one, half after a 200-step untimed run; each is printed to stderr and the
first is returned (so the JSON line is bench.py's usual one).  bench_data is wrapped to load enough batches.
Usage: python scripts/diag/bench_windows.py [bench args]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

WINDOWS = 6
_orig_data, _orig_region = bench.bench_data, bench.timed_region


def data(world, rank, batch, total_steps, mode="hard"):
    return _orig_data(world, rank, batch, total_steps + WINDOWS * 220, mode)


def region(ctx, tr, run, steps, cuda_sync, clock=time.perf_counter):
    first = _orig_region(ctx, tr, run, steps, cuda_sync, clock)
    print(f"window 0 (bench): {first / steps * 1e3:.4f} ms/step", file=sys.stderr, flush=True)
    for i in range(1, WINDOWS + 1):
        if i > WINDOWS // 2:
            run(200)
        t = _orig_region(ctx, tr, run, steps, cuda_sync, clock)
        print(f"window {i} ({'after 200 steps' if i > WINDOWS // 2 else 'back to back'}): {t / steps * 1e3:.4f} ms/step",
              file=sys.stderr, flush=True)
    return first


bench.bench_data, bench.timed_region = data, region
sys.exit(bench.main(sys.argv[1:]))
