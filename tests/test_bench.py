"""bench.py contract on CPU: ``--gpus N`` starts N ranks itself (no torchrun environment) and
relays exactly one JSON line with ``n_gpus == N``; a WORLD_SIZE / --gpus mismatch is an error.
The ``--dry-run`` mode runs the same launcher, rendezvous (gloo, 127.0.0.1) and halo-exchange
path on the numpy backend, so this needs no GPU."""

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=REPO)


@pytest.mark.parametrize("gpus,decomp", [(1, "jstrips"), (2, "jstrips"), (2, "2d"), (3, "jstrips"),
                                         (4, "jstrips"), (4, "2d"), (8, "jstrips"), (8, "2d")])
def test_bench_launcher_dry_run(gpus, decomp):
    """The driver's 1/2/4/8-rank command lines, rehearsed on the CPU (gloo, numpy backend, a
    64x32x8 tile per rank): one JSON line with the whole N-rank record, C5 leg included."""
    res = _run(["--dry-run", "--gpus", str(gpus), "--steps", "2", "--warmup", "1", "--decomp", decomp],
               timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, res.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == gpus
    assert rec["dry_run"] is True
    assert rec["steps"] == 2 and rec["warmup"] == 1
    gi, gj, _ = rec["config"]["global_domain"]
    assert gi * gj == 64 * 32 * gpus and rec["config"]["domain_per_gpu"][:2] == [64, 32]
    assert rec["hbm_estimate"]["peak_gb"] >= rec["hbm_estimate"]["fields_gb"] > 0
    if gpus > 1:
        assert rec["config"]["parallelism"].startswith("ij-")
        # the line names what moved the halos (the dry run's gloo, RCCL on the GPU nodes)
        assert rec["config"]["workload"].endswith("gloo (host-staged) halo 2"), rec["config"]["workload"]
        if decomp == "2d":  # a balanced process grid: 2x2 at 4 ranks, 2x4 at 8
            want = {2: "1x2", 4: "2x2", 8: "2x4"}.get(gpus)
            if want is not None:
                assert rec["config"]["parallelism"] == f"ij-tiles{want}", rec["config"]
        # the N>1 line explains itself
        d = rec["dist"]
        assert d["world_size"] == gpus
        assert [r["rank"] for r in d["ranks"]] == list(range(gpus))
        assert "rccl_version" in d
        for k in ("step_ms", "plain_ms_per_step", "plain_kernel_ms", "exchange_overhead"):
            assert k in d
        assert isinstance(d["exchange_overhead"], float)
        if decomp == "jstrips":  # real peers: the interior is gated on the pack
            assert d["halo_schedule"]["gate"] is True and d["halo_schedule"]["strips"] == "halo stream"
        assert rec["roofline"]["traffic"] is None and "halo step" in rec["roofline"]["traffic_source"]
        assert "step_ms" in rec["roofline"] and "kernel_ms" not in rec["roofline"]
        # C5 (the f32 tile) through the same N-rank path, whole-job cells/s
        c5 = rec["extra_configs"]["hdiff_f32"]
        assert "error" not in c5, c5
        assert c5["n_gpus"] == gpus and c5["global_domain"][0] * c5["global_domain"][1] == 64 * 32 * gpus
        assert c5["Mcells_s"] > 0 and c5["scaling"] == "weak"
        # the link probe ran before the headline: one face-sized message to and from each peer
        lp = d["link_probe"]
        assert [r["rank"] for r in lp["ranks"]] == list(range(gpus)) and lp["all_payloads_ok"]
        for r in lp["ranks"]:
            assert r["bytes_per_message"] == 10_485_760 and r["peers"] and r["rank"] not in r["peers"]
            assert r["ms"] > 0 and r["GBps_per_link_each_way"] > 0
            if decomp == "jstrips":
                assert r["peers"] == [p for p in (r["rank"] - 1, r["rank"] + 1) if 0 <= p < gpus]
        assert lp["min_GBps_per_link"] > 0
    else:
        assert "dist" not in rec
        # C2 and C4 carry their own cpu_ifirst-equivalent figure (BASELINE configs[1])
        for cfg in ("lap5", "tridiag"):
            cb = rec["extra_configs"][cfg]["cpu_baseline"]
            assert "error" not in cb, cb
            assert cb["value"] > 0 and cb["unit"] == "Mcells/s" and cb["ms_per_call"] > 0
            assert cb["cores"] >= 1 and cb["kind"] == "port" and cb["sample"]
            assert cb["dry_run_domain"] == [64, 32, 8]
    for key in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "scaling", "roofline", "config"):
        assert key in rec


def test_rank_setup_timeout_names_the_phase():
    """A rank that cannot finish process-group set-up exits non-zero with its last phase (here:
    rank 1 of a 2-rank rendezvous never starts, so rank 0 waits in init_process_group)."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    res = _run(["--dry-run", "--gpus", "2", "--steps", "1", "--warmup", "0"],
               env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                          "MASTER_PORT": str(port), "GTMI_DIST_SETUP_TIMEOUT": "5", "GTMI_DIST_TIMEOUT": "120"},
               timeout=120)
    assert res.returncode == 3, (res.returncode, res.stderr[-2000:])
    assert "no progress past phase 'init_process_group'" in res.stderr


def test_bench_world_size_mismatch_is_an_error():
    res = _run(["--dry-run", "--gpus", "2"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert res.returncode == 2
    assert "WORLD_SIZE" in res.stderr


@pytest.mark.gpu
def test_bench_gpu_line_with_placement_tuning():
    """The real N=1 line on the GPU (small config): one JSON line, roofline within [0, 1], and the
    written field placed by measurement with every buffer set's time recorded (set 0 = the first
    allocation, the untuned time)."""
    res = _run(["--config", "lap5", "--steps", "5", "--warmup", "2", "--no-extra", "--no-cpu-baseline",
                "--sustain", "0", "--placement-candidates", "2"], timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, res.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1 and rec["dtype"] == "f64" and rec["unit"] == "Mcells/s"
    assert 0.0 < rec["roofline"]["frac"] <= 1.0
    p = rec["placement"]
    assert p["written"] == ["out_field"] and len(p["candidates_ms"]) == 3
    assert p["tuned_ms"] == min(p["candidates_ms"]) == p["candidates_ms"][p["chosen"]]
    assert p["untuned_ms"] == p["candidates_ms"][0] and p["in_place"]
    assert rec["full_call"]["overhead_vs"] == "kernel_ms"
    r = rec["roofline"]
    assert 0.0 < r["frac_untuned"] <= 1.0 and r["kernel_ms_untuned"] > 0


@pytest.mark.gpu
def test_bench_halo_selfcomm_link_probe():
    """One GPU as its own periodic neighbour through RCCL (``--halo-selfcomm``): the line carries
    the link probe of the one rank (peer = itself, payload intact) next to the halo A/B."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    res = _run(["--config", "lap5", "--steps", "3", "--warmup", "1", "--no-extra", "--no-cpu-baseline", "--sustain", "0",
                "--placement-candidates", "0", "--halo-selfcomm"],
               env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                          "MASTER_PORT": str(port)}, timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    rec = json.loads([ln for ln in res.stdout.splitlines() if ln.strip()][-1])
    lp = rec["dist"]["link_probe"]
    (r0,) = lp["ranks"]
    assert r0["peers"] == [0] and r0["payload_ok"] and r0["GBps_per_link_each_way"] > 0
    assert rec["halo_ab"]["overhead"] > -0.5
    # one GPU as its own neighbour keeps the ungated schedule (auto gate: real peers only)
    assert rec["halo_ab"]["halo_schedule"]["gate"] is False
