"""bench.py's host-side pieces without a GPU: the CPU baseline runs the reference's
update_checksums() (oracle/_ref, compiled from /root/reference) on every CPU of the process's
affinity set by default (SURVEY.md §8d "all host cores"), one pinned std::thread each, interleaved
across NUMA nodes; its line states the cores used, the allotment and the cgroup's CPU quota."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_allotted_cpus_interleave_the_affinity_set():
    import bench
    cpus = bench.allotted_cpus()
    assert sorted(cpus) == sorted(os.sched_getaffinity(0))


def test_cpu_baseline_defaults_to_every_allotted_cpu():
    import bench
    import oracle
    oracle.build()
    r = bench.cpu_baseline(0, 0, 0.2, "update", 0.1, 0.1)  # C0: 1024 x 64 B, a fraction of a second
    assert r["runs"][-1]["threads"] == len(os.sched_getaffinity(0)) == r["nproc"]
    assert r["value"] > 0 and r["one_core"] > 0
    assert r["kind"] == ("reference" if oracle.ref_available() else "port")
    assert "cgroup_cpu_quota" in r and "numa_nodes" in r


def test_bench_defaults():
    """No flags: N = 1, config C1 (BASELINE configs[1]), the CPU baseline on every allotted CPU."""
    import bench
    a = bench.make_parser().parse_args([])
    assert (a.gpus, a.config, a.packets, a.align, a.cpu_threads) == (1, 1, 0, 128, 0)
    assert not a.no_cpu and not a.no_c4 and a.op == "update"


def test_cpu_baseline_reports_its_fastest_thread_count(monkeypatch):
    """the reported baseline is the best rate measured, not the slowest; with a
    cgroup quota below the affinity set both thread counts run and the faster one is `value`."""
    import bench
    import oracle
    oracle.build()
    ncpu = len(os.sched_getaffinity(0))
    if ncpu > 2:  # pretend the cgroup grants 2 CPUs of run time
        monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: 2.0)
    r = bench.cpu_baseline(0, 0, 0.2, "update", 0.1, 0.1)
    rates = {x["threads"]: x["value"] for x in r["runs"]}
    assert r["value"] == max(rates.values())
    assert rates[r["cores"]] == r["value"]
    if ncpu > 2:
        assert set(rates) == {ncpu, 2}
