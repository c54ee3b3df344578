"""Per-rank host CPU plan for the one-process-per-GPU runs (bench.py --gpus N,
localGraph under torch.distributed.run; SVscope.py:158-165 sizes its Pool the
same way, per process).

Each rank's engine runs a fork-join pool for its host work (feature
selection, ward linkage, record assembly; csrc/svs_threadpool.cpp).  Sized
from the whole machine, eight ranks would each start 16 threads on a job that
owns 16 cores.  The plan therefore splits the job's CPUs between the ranks of
this node:

  * the job's CPUs are its affinity mask, capped by the job's CPU share when
    the environment states one (OMP_NUM_THREADS: the GPU boxes set it to the
    share);
  * rank r of LOCAL_WORLD_SIZE W gets the r-th contiguous slice of the
    affinity mask (contiguous CPU ids share a NUMA node on the MI355X hosts,
    so each rank's threads stay on one socket) and max(2, share // W) pool
    threads, at most 16.

``apply()`` pins the process to its slice and exports SVS_HOST_THREADS, which
the library reads when a context is created (svs_abi.cpp host_threads), so it
must run before the first context.  A caller-set SVS_HOST_THREADS wins.
"""
import os

MAX_THREADS = 16


def job_cpus():
    try:
        return sorted(os.sched_getaffinity(0))
    except AttributeError:
        return list(range(os.cpu_count() or 1))


def job_share(cpus):
    share = os.environ.get("OMP_NUM_THREADS", "")
    n = len(cpus)
    if share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def rank_cpu_plan(local_rank, local_world, cpus=None, share=None):
    """(cpus of this rank, pool threads) for rank ``local_rank`` of
    ``local_world`` ranks on this node."""
    cpus = list(cpus) if cpus is not None else job_cpus()
    share = share if share is not None else job_share(cpus)
    w = max(1, int(local_world))
    r = min(max(0, int(local_rank)), w - 1)
    if w == 1:
        mine = cpus
    else:
        lo, hi = r * len(cpus) // w, (r + 1) * len(cpus) // w
        mine = cpus[lo:hi] or cpus[r % len(cpus):r % len(cpus) + 1]
    threads = max(2, min(MAX_THREADS, share // w))
    return mine, threads


def apply(local_rank=None, local_world=None):
    """Pins this process to its slice and sets SVS_HOST_THREADS (unless the
    caller set it).  Returns the pool size the library will use."""
    if local_rank is None:
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if local_world is None:
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    mine, threads = rank_cpu_plan(local_rank, local_world)
    if int(local_world) > 1 and hasattr(os, "sched_setaffinity"):
        try:
            os.sched_setaffinity(0, mine)
        except OSError:
            pass
    if not os.environ.get("SVS_HOST_THREADS"):
        os.environ["SVS_HOST_THREADS"] = str(threads)
    return int(os.environ["SVS_HOST_THREADS"])
