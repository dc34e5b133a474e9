"""Host facts shared by the GPU tests (no GPU needed)."""
import os


def host_threads() -> int:
    """The host threads this process may use (affinity, cgroup quota, OMP_NUM_THREADS)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, min(n, 16))
