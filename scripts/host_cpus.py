"""CPU capacity of this host as a process sees it (JSON on stdout): logical
CPUs (nproc), the affinity mask, the cgroup CPU quota and the CPU model.
bench.py uses the same function for its cpu_baseline."""
import json
import os


def host_cpu_info():
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = info["nproc"]
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):  # cgroup v2: "<quota> <period>" or "max <period>"
        try:
            with open(path) as f:
                q, p = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(p)
        except (OSError, ValueError):
            pass
    if quota is None:  # cgroup v1
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                p = int(f.read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    info["cgroup_cpu_quota"] = quota
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    info["cpu_model"] = model
    info["omp_num_threads"] = os.environ.get("OMP_NUM_THREADS")
    # CPUs this process can keep busy: the affinity mask, capped by the
    # cgroup quota (the GPU box gives one GPU's job a 16-CPU quota of a
    # 256-CPU host: threads beyond it are throttled, not added)
    usable = info["affinity"] or 1
    if quota is not None:
        usable = max(1, min(usable, int(quota)))
    info["usable"] = usable
    return info


if __name__ == "__main__":
    print(json.dumps(host_cpu_info()))
