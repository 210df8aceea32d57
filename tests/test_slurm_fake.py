"""T2b: the SLURM entrypoint and the CI submit/poll script against fake SLURM commands
(tests/fake_slurm: srun/sbatch/squeue/scontrol/scancel shims; no cluster, no GPU)."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIMS = os.path.join(ROOT, "tests", "fake_slurm")
pytestmark = pytest.mark.slow


def _env(tmp_path, **extra):
    e = dict(os.environ)
    e.update({"PATH": SHIMS + os.pathsep + e["PATH"], "FAKE_SLURM_DIR": str(tmp_path), "DGT_WORKDIR": ROOT,
              "DGT_LOG_DIR": str(tmp_path / "logs"), "DGT_IMAGE": "unused.sqsh", "GPUS_PER_NODE": "2",
              "NNODES": "1", "DGT_QUIET": "1", "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": "",
              "DGT_BACKEND": "gloo"})
    e.update(extra)
    return e


def _run_sbatch(tmp_path, train_args):
    env = _env(tmp_path, SLURM_JOB_ID="4242", SLURM_JOB_NODELIST="mi355x-[001-001]", SLURM_SUBMIT_DIR=str(tmp_path),
               SLURM_JOB_NUM_NODES="1", TRAIN_ARGS=train_args)
    return subprocess.run(["bash", os.path.join(ROOT, "slurm_train.sbatch")], cwd=tmp_path, env=env,
                          capture_output=True, text=True, timeout=300)


def test_sbatch_success_writes_status_and_health(tmp_path):
    r = _run_sbatch(tmp_path, "--epochs 1 --no-save")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert (tmp_path / "job_status.txt").read_text().strip() == "success"
    assert "✅ job success" in r.stdout
    assert "Epoch  1 finished. Avg loss: 0.5126" in r.stdout  # 2 ranks (GPUS_PER_NODE=2)
    rep = json.loads((tmp_path / "logs" / "health_job4242_node0.json").read_text())
    assert "gpu" in rep and rep["node"] == 0


def test_sbatch_failure_propagates(tmp_path):
    r = _run_sbatch(tmp_path, "--epochs 1 --no-save --fail-at 0:end")
    assert r.returncode != 0
    assert (tmp_path / "job_status.txt").read_text().strip() == "fail"
    assert "❌ job fail" in r.stdout


@pytest.mark.parametrize("fail,want_rc", [(False, 0), (True, 1)])
def test_ci_submit_and_wait(tmp_path, fail, want_rc):
    shutil.copy(os.path.join(ROOT, "slurm_train.sbatch"), tmp_path)
    env = _env(tmp_path, DGT_POLL_INTERVAL="1", DGT_POLL_MAX="240", DGT_STATUS_POLL_INTERVAL="1",
               FAKE_SLURM_GPUS="2", FAKE_SLURM_NODES="1",
               TRAIN_ARGS="--epochs 1 --no-save" + (" --fail-at 1:end" if fail else ""))
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "slurm_submit_and_wait.sh"), str(tmp_path)],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == want_rc, r.stdout[-3000:] + r.stderr[-2000:]
    sub = (tmp_path / "slurm_train.submit.sbatch").read_text()
    assert "#SBATCH --nodes=1" in sub and "#SBATCH --gres=gpu:2" in sub
    assert "Submitted batch job" in r.stdout


def test_ci_submit_timeout_cancels(tmp_path):
    shutil.copy(os.path.join(ROOT, "slurm_train.sbatch"), tmp_path)
    env = _env(tmp_path, DGT_POLL_INTERVAL="1", DGT_POLL_MAX="2", FAKE_SLURM_GPUS="2",
               TRAIN_ARGS="--epochs 1 --no-save --fail-at 0:1:hang")
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "slurm_submit_and_wait.sh"), str(tmp_path)],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 124, r.stdout[-2000:]


def test_ci_workflow_structure():
    """The CI pipeline keeps the reference's shape (build -> SLURM acceptance test -> publish only on
    success, .github/workflows/distributed-gpu-test-ci.yaml:18-231) plus a CPU unit-test gate."""
    import yaml
    wf = yaml.safe_load(open(os.path.join(ROOT, ".github", "workflows", "distributed-gpu-test-ci.yaml")))
    jobs = wf["jobs"]
    assert {"unit-tests", "build", "test-on-slurm", "publish"} <= set(jobs)
    needs = lambda j: set([jobs[j]["needs"]] if isinstance(jobs[j].get("needs"), str) else jobs[j].get("needs", []))
    assert "build" in needs("test-on-slurm")
    assert {"build", "test-on-slurm"} <= needs("publish")
    text = open(os.path.join(ROOT, ".github", "workflows", "distributed-gpu-test-ci.yaml")).read()
    assert "rocm" in text.lower() and "nvidia" not in text.lower()
