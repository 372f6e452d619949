"""bench.py end to end at small sizes: the multi-rank launcher (--gpus N without a launcher
starts the ranks itself), the post-timing oracle checks of the timed output, the gathered
array check, and the probe's full oracle comparison.  The GPU tests run bench.py as a child
process on the one-GPU box (two gloo ranks share the device)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, env=None, timeout=400):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True,
                       text=True, timeout=timeout, env=e, cwd=ROOT)
    return r


def last_json(r):
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads(lines[-1])


def test_bench_refuses_world_mismatch():
    """Under a launcher the world size must equal --gpus (a mislaunched scaling run must not
    report n_gpus: 1)."""
    r = run_bench("--gpus", "2", env={"WORLD_SIZE": "1"}, timeout=120)
    assert r.returncode != 0
    assert "--gpus 2 but WORLD_SIZE=1" in r.stderr


SMALL = ["--steps", "3", "--warmup", "1", "--ramp-ms", "0", "--no-e2e", "--no-cpu-baseline"]


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["bloom10", "vqf12"])
def test_bench_two_ranks_gloo(workload):
    """--gpus 2 with no launcher: two ranks (sharing the box's one GPU over gloo), n_gpus 2,
    every rank's sampled leaves equal the oracle, and rank 0 finds the all-gathered array
    equal to a single-process build of all leaves."""
    r = run_bench("--gpus", "2", "--backend", "gloo", "--keys-per-gpu", "2000000",
                  "--workload", workload, *SMALL)
    assert r.returncode == 0, r.stderr[-4000:]
    d = last_json(r)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["config"]["total_keys"] == 4_000_000
    assert d["verified"] is True and d["verify"]["all_ranks_ok"] is True
    assert d["gather_verified"] is True
    assert d["allgather_ms"] > 0


@pytest.mark.gpu
def test_bench_two_ranks_nccl():
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("RCCL needs one GPU per rank")
    r = run_bench("--gpus", "2", "--keys-per-gpu", "2000000", *SMALL)
    assert r.returncode == 0, r.stderr[-4000:]
    d = last_json(r)
    assert d["n_gpus"] == 2 and d["gather_verified"] is True and d["verified"] is True


@pytest.mark.gpu
def test_bench_strong_scaling_two_ranks():
    """--total-keys (config 5's form): one checkpoint split by leaf range; the last rank
    holds fewer leaves, the gathered array still equals the single-process build."""
    r = run_bench("--gpus", "2", "--backend", "gloo", "--workload", "bloom12",
                  "--total-keys", "3000001", *SMALL)
    assert r.returncode == 0, r.stderr[-4000:]
    d = last_json(r)
    assert d["scaling"] == "strong" and d["n_gpus"] == 2
    assert d["gather_verified"] is True and d["verified"] is True


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["probe10", "probe_vqf12"])
def test_bench_probe_matches_oracle(workload):
    """Config 4's check at a small size: every answer equals the oracle's over the GPU-built
    filter, so the FPRs are equal; the probe line carries a CPU baseline."""
    r = run_bench("--workload", workload, "--keys-per-gpu", "1000000", "--steps", "3",
                  "--warmup", "1", "--ramp-ms", "0", "--no-e2e")
    assert r.returncode == 0, r.stderr[-4000:]
    d = last_json(r)
    p = d["probe"]
    assert p["results_equal_oracle"] is True and d["verified"] is True
    assert p["fpr_oracle"] == p["false_positive_rate"]
    assert d["cpu_baseline"] and d["cpu_baseline"]["value"] > 0


@pytest.mark.gpu
def test_bench_single_gpu_line():
    """The default line's shape at a small size: verified sample, batch-size sweep, a CPU
    baseline with the host's CPU share stated."""
    r = run_bench("--keys-per-gpu", "3000000", "--steps", "3", "--warmup", "1", "--ramp-ms", "0",
                  "--no-e2e", "--sweep")
    assert r.returncode == 0, r.stderr[-4000:]
    d = last_json(r)
    assert d["n_gpus"] == 1 and d["verified"] is True
    v = d["verify"]   # every leaf, not a sample, and the device keys themselves
    assert v["leaves_checked"] == v["of_leaves"] == 184 and v["keys_equal_oracle"] is True
    assert [row["leaves"] for row in d["batch_sweep"]] == [64, 184]   # sizes below the batch
    b = d["cpu_baseline"]
    assert b["cores"] >= 1 and "host" in b and b["value"] > 0


@pytest.mark.gpu
def test_bench_two_ranks_gloo_host_legs():
    """N > 1 lines carry the north star's host figures: every rank runs its own end-to-end
    leg (its pages back to host page memory over its own link) at the same time, and rank 0
    times the CPU baseline after the other ranks have left."""
    r = run_bench("--gpus", "2", "--backend", "gloo", "--keys-per-gpu", "2000000",
                  "--steps", "3", "--warmup", "1", "--ramp-ms", "0", "--cpu-threads", "4")
    assert r.returncode == 0, r.stderr[-4000:]
    d = last_json(r)
    assert d["n_gpus"] == 2 and d["verified"] is True and d["gather_verified"] is True
    e = d["e2e_pcie_inclusive"]
    assert e["ranks"] == 2 and e["mkeys_s"] > 0 and e["from_key_views"]["mkeys_s"] > 0
    b = d["cpu_baseline"]
    assert b and b["value"] > 0 and b["cores"] >= 1 and "rank 0" in b["note"]
    assert d["allgather_bytes_in_per_gpu"] > 0
    assert d["build_plus_allgather_pipelined"]["ms_per_step"] > 0


def run_launched(*args, timeout=400):
    """bench.py under torch.distributed.run with one rank: the process-group code paths
    (RCCL init bound to the device, device all-reduces, the all-gather) at world size 1."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", *args]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e, cwd=ROOT)


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["bloom10", "bloom12hash"])
def test_bench_nccl_world1(workload):
    """The RCCL path before any 8-GPU run: init_process_group("nccl", device_id=...), the
    float64 / int32 all-reduces on the device, all_gather_into_tensor of the filter array, and
    (bloom12hash) the device all_to_all_single of the routed keys."""
    r = run_launched("--workload", workload, "--keys-per-gpu", "2000000", *SMALL)
    assert r.returncode == 0, r.stderr[-4000:]
    d = last_json(r)
    assert d["n_gpus"] == 1 and d["config"]["backend"] == "nccl" and d["verified"] is True
    if workload == "bloom10":
        assert d["allgather_ms"] > 0 and d["gather_verified"] is True
    else:   # the pipelined step: route -> part builds -> in-place all-gather of every round
        assert d["verify"]["equal_to_oracle"] and d["verify"]["header_ok"]
        assert d["config"]["allgather_in_step"] is True
        assert d["step_breakdown_rank0_ms"]["allgather"] > 0
        assert d["route_plan"]["overflow_lost"] is False


@pytest.mark.gpu
@pytest.mark.parametrize("workload,extra", [("bloom10", ["--keys-per-gpu", "2000000"]),
                                            ("vqf12", ["--keys-per-gpu", "2000000"]),
                                            ("bloom12", ["--total-keys", "3000001"])])
def test_bench_pipelined_gather_gloo(workload, extra):
    """--chunks: two gloo ranks build their block-cyclic rounds and all-gather each round on
    the communication stream while the next builds; rank 0 finds the gathered array equal to
    a one-GPU build of every leaf (strong scaling: ragged rounds, an empty last slot)."""
    r = run_bench("--gpus", "2", "--backend", "gloo", "--workload", workload, "--chunks", "3",
                  *extra, *SMALL)
    assert r.returncode == 0, r.stderr[-4000:]
    d = last_json(r)
    assert d["n_gpus"] == 2 and d["gather_verified"] is True
    assert d["config"]["rounds"] == 3 and d["comm"]["world_size"] == 2
    b = d["breakdown_ms"]
    assert b["build_only"] > 0 and b["gather_only"] > 0 and b["pipelined"] > 0


@pytest.mark.gpu
def test_bench_pipelined_gather_nccl_world1():
    """The same step over RCCL at world size 1: all_gather_into_tensor per round on the
    communication stream, the gathered array checked against a one-GPU build."""
    r = run_launched("--workload", "bloom10", "--keys-per-gpu", "2000000", "--chunks", "4", *SMALL)
    assert r.returncode == 0, r.stderr[-4000:]
    d = last_json(r)
    assert d["n_gpus"] == 1 and d["config"]["backend"] == "nccl" and d["gather_verified"] is True
    assert d["config"]["rounds"] == 4


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["probe10", "probe_vqf12"])
def test_bench_probe_full_size(workload):
    """Config 4 at its own size in the GPU suite: 200M shuffled hit/miss lookups against the
    100M-key build, every answer equal to the oracle's over the GPU-built filter bytes, so the
    FPRs are equal; no false negatives."""
    r = run_bench("--workload", workload, "--steps", "3", "--warmup", "1", "--ramp-ms", "0",
                  "--no-e2e", "--no-cpu-baseline", timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    d = last_json(r)
    p = d["probe"]
    assert p["lookups"] == 200_000_000 and p["hits_all_true"] is True
    assert p["results_equal_oracle"] is True and d["verified"] is True
    assert p["fpr_oracle"] == p["false_positive_rate"]
