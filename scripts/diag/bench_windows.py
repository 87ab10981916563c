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
if os.environ.get("HIP_SCHED"):  # device schedule flag before any HIP context: 1 spin, 2 yield, 4 blocking sync
    import ctypes
    import glob
    import torch  # (its bundled HIP runtime is the one every later call uses; importing does not create a context)
    _lib = (glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so*")) or ["libamdhip64.so"])[0]
    _hip = ctypes.CDLL(_lib)
    print(f"hipSetDeviceFlags({os.environ['HIP_SCHED']}) -> {_hip.hipSetDeviceFlags(int(os.environ['HIP_SCHED']))}",
          file=sys.stderr, flush=True)
import bench  # noqa: E402

WINDOWS = 6
SWEEP = os.environ.get("WINDOW_SWEEP") == "1"  # windows of 10..160 steps: fixed cost per window vs per step
SIZES = (10, 20, 40, 80, 160)
_orig_data, _orig_region = bench.bench_data, bench.timed_region


def data(world, rank, batch, total_steps, mode="hard"):
    extra = 3 * sum(SIZES) + 20 if SWEEP else WINDOWS * 220
    return _orig_data(world, rank, batch, total_steps + extra, mode)


def region(ctx, tr, run, steps, cuda_sync, clock=time.perf_counter):
    first = _orig_region(ctx, tr, run, steps, cuda_sync, clock)
    if SWEEP:
        print(f"window 0 (bench): {first / steps * 1e3:.4f} ms/step", file=sys.stderr, flush=True)
        pts = []
        for rep in range(3):
            for n in SIZES:
                t = _orig_region(ctx, tr, run, n, cuda_sync, clock)
                pts.append((n, t))
                print(f"sweep rep {rep} steps {n}: {t * 1e3:.4f} ms total, {t / n * 1e3:.4f} ms/step", file=sys.stderr,
                      flush=True)
        xs = [n for n, _ in pts]
        ys = [t for _, t in pts]
        mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
        b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
        a = my - b * mx
        print(f"fit: window = {a * 1e6:.1f} us + {b * 1e6:.2f} us/step", file=sys.stderr, flush=True)
        return first
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
