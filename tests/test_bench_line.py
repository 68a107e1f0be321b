"""CPU: bench.py's line assembly at N > 1 (no GPU touched) — the line the driver's 8-GPU
scaling run prints carries, at every GPU count, the reference CPU baseline timed in the same
run and the roofline fraction over all N devices (north_star: "report Mpps at each count as
absolute numbers and as a fraction of the HBM-read roofline, next to the reference CPU
parser+filter timed on the node's own host cores (core count stated) in the same run").

The per-rank results are stubs of what bench.measure() gathers from every rank."""
import argparse
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _ranks(world, algo=1.9e9, main_ms=0.33, step_s=0.34e-3):
    # rank r a little slower than rank 0: the aggregate uses the slowest one
    return [{"algo": algo, "main_ms": main_ms * (1 + 0.01 * r), "step_s": step_s * (1 + 0.01 * r), "n": 1 << 24}
            for r in range(world)]


def _entry(world, scaling="weak"):
    ranks = _ranks(world)
    return {"workload": "stub", "value": 1.0, "unit": "Mpps", "ms_per_step": 0.34, "scaling": scaling,
            "packets_per_gpu": 1 << 24, "packets_total": (1 << 24) * world, "pass_fraction": 0.1,
            "roofline": {"frac": 0.7}, "roofline_aggregate": bench.aggregate_roofline(ranks, world),
            "timing": {}, "per_rank": [{"rank": r} for r in range(world)]}


@pytest.mark.parametrize("world", [1, 2, 8])
def test_aggregate_roofline_sums_bytes_over_slowest_rank(world):
    ranks = _ranks(world)
    agg = bench.aggregate_roofline(ranks, world)
    slowest_ms = max(r["main_ms"] for r in ranks)
    want = world * 1.9e9 / (slowest_ms * 1e-3) / 1e9
    assert agg["devices"] == world and agg["peak"] == world * bench.HBM_PEAK_GBS
    assert agg["achieved"] == pytest.approx(want, abs=0.1)
    assert agg["frac"] == pytest.approx(want / (world * bench.HBM_PEAK_GBS), abs=1e-4)
    slowest_step = max(r["step_s"] for r in ranks)
    assert agg["frac_step"] == pytest.approx(world * 1.9e9 / slowest_step / 1e9 / (world * bench.HBM_PEAK_GBS),
                                             abs=1e-4)
    assert agg["frac_step"] <= agg["frac"]


def test_aggregate_equals_single_device_roofline_at_n1():
    r = _ranks(1)[0]
    agg = bench.aggregate_roofline([r], 1)
    assert agg["frac"] == pytest.approx(r["algo"] / (r["main_ms"] * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, abs=1e-4)


def test_two_rank_line_carries_cpu_baseline_and_aggregate_frac():
    world = 2
    results = {"__head__": _entry(world), "c3": _entry(world), "c3_strong": _entry(world, "strong")}
    samples = {k: (("frames", "desc"), {"filters": [1], "parse": True}) for k in results}
    calls = []

    def timer(sample, wl, seconds, cpus):
        calls.append(seconds)
        return {"value": 9.5, "unit": "Mpps", "cores": cpus["threads"], "kind": "reference", "sample": "stub"}

    cpus = {"model": "stub", "affinity_cpus": 16, "cgroup_quota_cpus": None, "threads": 16}
    bench.attach_cpu_baselines(results, samples, cpus, world, timer, 5.0)
    # timed once for the headline and once for c3; c3_strong quotes c3's (same capture, seed)
    assert calls == [5.0, 5.0]
    args = argparse.Namespace(steps=20, warmup=5)
    line = bench.build_line(results, args, world, {"devices_distinct": 2})
    assert line["n_gpus"] == 2
    cb = line["cpu_baseline"]
    assert cb and cb["kind"] == "reference" and cb["cores"] == 16 and cb["n_gpus_in_job"] == 2
    assert "other ranks waiting at a barrier" in cb["timed"]
    agg = line["roofline_aggregate"]
    assert agg["devices"] == 2 and 0 < agg["frac"] <= 1 and agg["peak"] == 2 * bench.HBM_PEAK_GBS
    assert line["configs"]["c3"]["cpu_baseline"]["value"] == 9.5
    assert line["configs"]["c3_strong"]["cpu_baseline"]["same_as"] == "configs.c3"
    assert line["configs"]["c3_strong"]["roofline_aggregate"]["devices"] == 2
    assert "__head__" not in line["configs"]


def test_headline_reports_all_affinity_threads_past_a_quota():
    results = {"__head__": _entry(1)}
    samples = {"__head__": (("frames", "desc"), {"filters": None, "parse": True})}
    seen = []

    def timer(sample, wl, seconds, cpus):
        seen.append(cpus["threads"])
        return {"value": 1.0, "unit": "Mpps", "cores": cpus["threads"], "kind": "port", "sample": "stub"}

    cpus = {"model": "stub", "affinity_cpus": 64, "cgroup_quota_cpus": 16.0, "threads": 16}
    bench.attach_cpu_baselines(results, samples, cpus, 1, timer, 4.0)
    assert seen == [16, 64]
    cb = results["__head__"]["cpu_baseline"]
    assert cb["all_affinity_threads"]["threads"] == 64 and cb["n_gpus_in_job"] == 1
    assert "barrier" not in cb["timed"]


def test_no_sample_means_no_baseline():
    results = {"__head__": _entry(2)}
    bench.attach_cpu_baselines(results, {"__head__": (None, {})}, {"affinity_cpus": 1, "threads": 1}, 2,
                               lambda *a: pytest.fail("timed without a sample"), 1.0)
    assert results["__head__"]["cpu_baseline"] is None


def test_group_ingest_runs_in_a_child_process_at_n_gt_1(monkeypatch):
    """At N > 1 rank 0 runs the group-ingest entry in a child process, so a failure there is
    reported in the line instead of ending rank 0. Here (no GPU) the child reports the skip."""
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.setenv(k, "0" if k != "WORLD_SIZE" else "2")   # the parent's rank env must not leak
    out = bench.group_ingest_isolated(2, 4096, timeout=240)
    assert out.get("process") == "child of rank 0", out
    assert "skipped" in out and "the job has 2" in out["skipped"]


def test_gloo_connection_lines_stay_off_stdout(tmp_path):
    """At N > 1 every rank's gloo init prints "[Gloo] Rank r is connected to ..." on stdout;
    bench.py points fd 1 at stderr around init_process_group so rank 0's stdout is the line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    code = ("import json, sys; sys.path.insert(0, %r); import bench, torch.distributed as d\n"
            "with bench.stdout_to_stderr(): d.init_process_group('gloo')\n"
            "d.barrier(); print(json.dumps({'rank': d.get_rank()}), flush=True); d.destroy_process_group()\n") % ROOT
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE="2")
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    for r, (out, err) in enumerate(outs):
        assert procs[r].returncode == 0, err
        assert out.strip().splitlines() == ['{"rank": %d}' % r], out
