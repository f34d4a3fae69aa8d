"""The bench.py driver contract on CPU (gloo): one JSON line from rank 0 with the metric /
config fields BASELINE.json names, for a single process and for torchrun with 2 ranks (the
driver's N > 1 launch line, minus the GPUs)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}


def _json_lines(out):
    recs = []
    for line in out.splitlines():
        line = line.strip()
        if line.startswith("{"):
            recs.append(json.loads(line))
    return recs


def _env():
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    return env


@pytest.mark.slow
def test_bench_single_process_json():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--tta", "0"],
                       cwd=ROOT, capture_output=True, text=True, timeout=600, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1
    rec = recs[0]
    assert KEYS <= rec.keys()
    assert rec["n_gpus"] == 1 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["higher_is_better"] is True and rec["scaling"] == "weak"
    assert rec["config"]["global_batch"] == 100
    assert rec["config"]["parallelism"] == "dp1-ps1-sync-flat"
    assert rec["config"]["variant"] == "mnist_sync_sharding (flat plan)"
    assert rec["prewarm"]["steps"] == 0  # CPU default; 100 untimed steps on a GPU


@pytest.mark.slow
def test_bench_torchrun_two_ranks_json(port):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--tta", "0.99", "--tta-steps", "2"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout  # rank 0 only
    rec = recs[0]
    assert KEYS <= rec.keys()
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 200
    assert rec["config"]["parallelism"] == "dp2-ps2-sync-flat"
    assert rec["config"]["plan"] == "flat"
    # whole-job aggregate: images/s = W * batch * steps / max-over-ranks time
    assert rec["value"] == pytest.approx(2 * 100 / (rec["ms_per_step"] / 1e3), rel=1e-3)
    # the reference's contiguous plan (BASELINE config 3) is timed on the same harness
    c = rec["plans"]["contiguous"]
    assert c["num_ps"] == 2 and c["ms_per_step"] > 0
    assert c["value"] == pytest.approx(2 * 100 / (c["ms_per_step"] / 1e3), rel=1e-3)
    # data semantics are labelled: the throughput window's per-worker
    # shards, and time to accuracy under both them and the reference's replicated batches
    assert rec["config"]["data_sharding"] == "stride"
    assert rec["time_to_acc"]["data_sharding"] == "stride"
    assert "steps_to_target" in rec["time_to_acc"]
    assert rec["time_to_acc_replicate"]["data_sharding"] == "replicate"
    assert rec["time_to_acc_replicate"]["steps_per_worker"] == 2
    # and on the hard synthetic set, under both protocols
    assert rec["time_to_acc_hard"]["data"].startswith("synthetic-hard")
    assert rec["time_to_acc_hard_replicate"]["data_sharding"] == "replicate"


@pytest.mark.slow
def test_bench_torchrun_exchange_ab_checks_replicas(port):
    """The W > 1 data-plane A/B (RCCL vs xGMI on a GPU node) on CPU ranks: two candidates of
    the same exchange must both pass the replica check (bitwise-equal parameters on every
    rank, finite, and identical to the first candidate's after the same steps)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--tta", "0", "--ab-steps", "2"]
    env = _env()
    env["DDL_AB_CANDIDATES"] = "rccl,rccl"
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    ab = recs[0]["exchange_ab"]
    assert ab["rccl"]["replicas_consistent"] is True
    assert ab["rccl"]["mean_diff_vs_rccl"] == 0.0
    assert "note" not in ab
