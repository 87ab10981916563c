"""Local multi-process launcher (``mpiexec -n N`` stand-in; no MPI in this image, survey Q19).

    python -m pytorch_ddp_mnist_amd.parallel.launch -n 4 [--style pmi|ompi|slurm|torch] -- \
        python3 mnist_pnetcdf_cpu_mp.py --parallel --wireup_method mpich

Spawns N children with the environment a real launcher would provide (PMI_RANK/PMI_SIZE for
MPICH/Hydra, OMPI_COMM_WORLD_* for Open MPI, SLURM_* for srun, RANK/WORLD_SIZE/LOCAL_RANK for
torchrun) plus MASTER_ADDR=127.0.0.1 and a free MASTER_PORT, so every reference wire-up method can
be exercised on one host.  Failure detection: the first child that exits non-zero (or a timeout)
terminates its siblings' process groups and the launcher exits with that child's code.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from collections import deque
from typing import List, Optional, Tuple


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def child_env(style: str, rank: int, n: int, port: int, base=None) -> dict:
    env = dict(os.environ if base is None else base)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["MASTER_ADDR"] = "127.0.0.1"
    env["MASTER_PORT"] = str(port)
    if style == "pmi":
        env.update(PMI_RANK=str(rank), PMI_SIZE=str(n), MPI_LOCALRANKID=str(rank))
    elif style == "ompi":
        env.update(OMPI_COMM_WORLD_RANK=str(rank), OMPI_COMM_WORLD_SIZE=str(n), OMPI_COMM_WORLD_LOCAL_RANK=str(rank),
                   PMIX_SERVER_URI2="pmix-server.1;tcp4://127.0.0.1:%d" % port)
        env.pop("MASTER_ADDR")
    elif style == "slurm":
        env.update(SLURM_PROCID=str(rank), SLURM_NTASKS=str(n), SLURM_LOCALID=str(rank), SLURM_JOB_NUM_NODES="1",
                   SLURM_TASKS_PER_NODE=str(n), SLURM_LAUNCH_NODE_IPADDR="127.0.0.1", SLURM_SRUN_COMM_PORT=str(port))
        env.pop("MASTER_ADDR")
        env.pop("MASTER_PORT")
    else:  # torch
        env.update(RANK=str(rank), WORLD_SIZE=str(n), LOCAL_RANK=str(rank))
    return env


def launch(cmd: List[str], n: int, style: str = "pmi", timeout: float = 0.0) -> int:
    port = free_port()
    procs = [subprocess.Popen(cmd, env=child_env(style, r, n, port), start_new_session=True) for r in range(n)]
    t0 = time.time()
    rc = 0
    try:
        while True:
            alive = 0
            for p in procs:
                code = p.poll()
                if code is None:
                    alive += 1
                elif code != 0 and rc == 0:
                    rc = code
            if rc != 0 or alive == 0:
                break
            if timeout and time.time() - t0 > timeout:
                rc = 124
                break
            time.sleep(0.05)
    finally:
        if rc != 0:
            for p in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
    return rc


_SINK_LOCK = threading.Lock()


def _pump(stream, sink, keep: Optional[list], prefix: str = "", tail: Optional[deque] = None, log=None) -> None:
    """Forward ``stream`` line by line (whole lines under one lock: ranks never interleave inside a line)."""
    for line in iter(stream.readline, ""):
        if keep is not None:
            keep.append(line)
        if tail is not None:
            tail.append(line)
        if log is not None:
            log.write(line)
            log.flush()
        with _SINK_LOCK:
            sink.write(prefix + line)
            sink.flush()
    stream.close()


def _exit_desc(code: Optional[int]) -> str:
    if code is None:
        return "still running (terminated by the launcher)"
    if code < 0:
        try:
            return f"killed by signal {signal.Signals(-code).name} ({128 - code})"
        except ValueError:
            return f"killed by signal {-code}"
    return f"exit code {code}"


def launch_relay(cmd: List[str], n: int, style: str = "torch", timeout: float = 0.0,
                 relay_rank: int = 0, extra_env: Optional[dict] = None,
                 log_dir: Optional[str] = None, tail_lines: int = 60) -> Tuple[int, List[str]]:
    """``launch`` for one-process-per-GPU jobs whose rank-``relay_rank`` stdout is the result.

    That rank's stdout is forwarded to ours (and returned as a list of lines); every other
    rank's stdout goes to our stderr, so exactly one rank can print to stdout.  Every rank's
    stderr is piped separately and forwarded to ours with a ``[rank r] `` prefix (whole lines),
    and -- with ``log_dir`` (or ``MNIST_AMD_RANK_LOG_DIR``) -- also written to
    ``log_dir/rank<r>.stderr``.  When the job fails, each rank's exit status (signal names
    included) and its last ``tail_lines`` stderr lines are printed as one block per rank, so the
    failing rank's own evidence (a native backtrace, a HIP error) is not lost in the other
    ranks' output.  The children start before this process touches a GPU (it never does).
    Exit code: the first non-zero child code, 124 on timeout, else 0; the surviving children
    are killed on failure.
    """
    port = free_port()
    log_dir = log_dir or os.environ.get("MNIST_AMD_RANK_LOG_DIR") or None
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
    procs, pumps, kept, tails, logs = [], [], [], [], []
    first_bad = None
    for r in range(n):
        env = child_env(style, r, n, port)
        env["LOCAL_WORLD_SIZE"] = str(n)
        env.update(extra_env or {})
        p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                             start_new_session=True)
        procs.append(p)
        tail = deque(maxlen=tail_lines)
        tails.append(tail)
        log = open(os.path.join(log_dir, f"rank{r}.stderr"), "w") if log_dir else None
        logs.append(log)
        for args in ((p.stdout, sys.stdout if r == relay_rank else sys.stderr, kept if r == relay_rank else None),
                     (p.stderr, sys.stderr, None, f"[rank {r}] ", tail, log)):
            th = threading.Thread(target=_pump, args=args, daemon=True)
            th.start()
            pumps.append(th)
    t0 = time.time()
    rc = 0
    # a SIGTERM to the launcher (e.g. `timeout`) must not orphan the ranks (they run in their own sessions)
    prev_term = None
    if threading.current_thread() is threading.main_thread():
        def _on_term(signum, frame):
            raise SystemExit(128 + signum)
        prev_term = signal.signal(signal.SIGTERM, _on_term)
    try:
        while True:
            alive = 0
            for i, p in enumerate(procs):
                code = p.poll()
                if code is None:
                    alive += 1
                elif code != 0 and rc == 0:
                    rc, first_bad = code, i
            if rc != 0 or alive == 0:
                break
            if timeout and time.time() - t0 > timeout:
                rc = 124
                sys.stderr.write(f"[launch] timeout after {timeout:.0f} s: terminating the ranks\n")
                break
            time.sleep(0.05)
    except BaseException:
        rc = rc or 143
        raise
    finally:
        if prev_term is not None:
            signal.signal(signal.SIGTERM, prev_term)
        codes = [p.poll() for p in procs]  # before the launcher terminates anyone
        if rc != 0:
            for p in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
        for th in pumps:
            th.join(timeout=5)
        for log in logs:
            if log is not None:
                log.close()
        if rc != 0:
            with _SINK_LOCK:
                for r in range(n):
                    mark = " <- first failure" if r == first_bad else ""
                    sys.stderr.write(f"==== [launch] rank {r}: {_exit_desc(codes[r])}{mark}; last stderr lines "
                                     f"({len(tails[r])}) ====\n")
                    sys.stderr.writelines(tails[r])
                sys.stderr.flush()
    return (rc if rc >= 0 else 128 - rc), kept


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-n", "--nproc", type=int, default=1)
    ap.add_argument("--style", choices=["pmi", "ompi", "slurm", "torch"], default="pmi")
    ap.add_argument("--timeout", type=float, default=0.0)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("no command")
    return launch(cmd, a.nproc, a.style, a.timeout)


if __name__ == "__main__":
    sys.exit(main())
