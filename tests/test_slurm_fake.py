"""T2b: the SLURM entrypoint and the CI submit/poll script against fake SLURM commands
(tests/fake_slurm: srun/sbatch/squeue/scontrol/scancel shims; no cluster, no GPU).

The fake ``srun`` emulates Pyxis: ``--container-image`` is a fake image directory built from the
repository's Dockerfile (``fake_image.build_fake_image``: its ENV, WORKDIR, COPY lines and build
step) and ``--container-mounts`` hides the image's files under the mount point.  Jobs are
submitted from a directory holding ONLY the files the CI workflow copies to the SLURM host
(``fake_image.stage_submit_dir`` reads the workflow's scp list), so a job that needs anything the
image does not provide fails here as it would on the cluster (missing #1).
Reference: slurm_train.sbatch:3-4,19-20,33-45 and .github/workflows/distributed-gpu-test-ci.yaml:64-73,107-181.
"""
import json
import os
import random
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIMS = os.path.join(ROOT, "tests", "fake_slurm")
sys.path.insert(0, SHIMS)
from fake_image import build_fake_image, ci_scp_files, stage_submit_dir  # noqa: E402

pytestmark = pytest.mark.slow


@pytest.fixture(scope="module")
def image(tmp_path_factory):
    d = tmp_path_factory.mktemp("image")
    build_fake_image(str(d))
    return d


def _env(tmp_path, image, **extra):
    e = dict(os.environ)
    for k in ("PYTHONPATH", "RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "DGT_HOME"):
        e.pop(k, None)
    e.update({"PATH": SHIMS + os.pathsep + e["PATH"], "FAKE_SLURM_DIR": str(tmp_path),
              "DGT_IMAGE": str(image), "GPUS_PER_NODE": "2", "NNODES": "1", "DGT_QUIET": "1",
              "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": "", "DGT_BACKEND": "gloo"})
    e.update(extra)
    return e


def _submit_dir(tmp_path):
    sub = tmp_path / "submit"
    sub.mkdir()
    stage_submit_dir(str(sub))
    return sub


def _run_sbatch(tmp_path, image, train_args, nodes=1, gpus=2):
    sub = _submit_dir(tmp_path)
    job = str(random.randint(1000, 19999))
    env = _env(tmp_path, image, SLURM_JOB_ID=job, SLURM_JOB_NODELIST=f"mi355x-[001-{nodes:03d}]",
               SLURM_SUBMIT_DIR=str(sub), SLURM_JOB_NUM_NODES=str(nodes), NNODES=str(nodes),
               GPUS_PER_NODE=str(gpus), TRAIN_ARGS=train_args)
    r = subprocess.run(["bash", str(sub / "slurm_train.sbatch")], cwd=sub, env=env, capture_output=True,
                       text=True, timeout=400)
    return r, sub, job


def test_fake_image_holds_the_framework_outside_the_mount(image):
    meta = json.load(open(image / ".fake_image.json"))
    home = meta["env"]["DGT_HOME"]
    assert home == "/opt/dgt" and meta["env"]["PYTHONPATH"] == home
    assert meta["workdir"] == "/workspace"
    base = image / home.lstrip("/")
    for f in ("train.py", "scripts/health.py", "distributed_gpu_test_amd/__init__.py", "configs/ds_zero1.json"):
        assert (base / f).exists(), f
    if os.path.exists(os.path.join(ROOT, "distributed_gpu_test_amd", "_C.so")):
        assert (base / "distributed_gpu_test_amd" / "_C.so").exists()
    if os.path.exists(os.path.join(ROOT, "build", "bin", "rccl_perf")):
        assert os.access(base / "build" / "bin" / "rccl_perf", os.X_OK)
    # nothing the job runs may live under the mount point
    assert not any((image / "workspace").iterdir())
    # the CI copies only login-node files; the job runs nothing from the submit dir
    assert set(ci_scp_files()) == {"slurm_train.sbatch", "scripts/slurm_submit_and_wait.sh"}


def test_mount_hides_an_image_installed_under_workspace(tmp_path):
    """The round-1 layout (package + _C.so under the image's /workspace, job runs /workspace/train.py
    from the mounted submit dir) dies with ModuleNotFoundError under the emulated mount; the same
    command against the current image works."""
    old_df = tmp_path / "Dockerfile.r1"
    old_df.write_text("FROM rocm/pytorch\nWORKDIR /workspace\n"
                      "COPY distributed_gpu_test_amd/ /workspace/distributed_gpu_test_amd/\n"
                      "COPY train.py /workspace/\nRUN python3 tools/build_ext.py -j 8\n")
    old_img = tmp_path / "old_image"
    build_fake_image(str(old_img), dockerfile=str(old_df))
    sub = tmp_path / "submit"
    sub.mkdir()
    shutil.copy(os.path.join(ROOT, "train.py"), sub)  # the round-1 CI copied train.py, not the package
    env = _env(tmp_path, old_img)
    cmd = ["srun", f"--container-image={old_img}", f"--container-mounts={sub}:/workspace",
           "python3", "/workspace/train.py", "--epochs", "1", "--no-save"]
    r = subprocess.run(cmd, cwd=sub, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "ModuleNotFoundError: No module named 'distributed_gpu_test_amd'" in r.stderr


def test_sbatch_success_writes_status_and_health(tmp_path, image):
    r, sub, job = _run_sbatch(tmp_path, image, "--epochs 1 --no-save")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert (sub / "job_status.txt").read_text().strip() == "success"
    assert "✅ job success" in r.stdout
    assert "Epoch  1 finished. Avg loss: 0.5126" in r.stdout  # 2 ranks (GPUS_PER_NODE=2)
    rep = json.loads((sub / "logs" / f"health_job{job}_node0.json").read_text())
    assert "gpu" in rep and rep["node"] == 0
    fw = rep["framework"]
    img_home = str(image / "opt" / "dgt")
    assert fw["dgt_home"] == img_home  # health.py ran from the image
    assert fw["package"] == os.path.join(img_home, "distributed_gpu_test_amd")
    if os.path.exists(os.path.join(ROOT, "build", "bin", "rccl_perf")):
        assert fw["rccl_perf"] == os.path.join(img_home, "build", "bin", "rccl_perf")
    if os.path.exists(os.path.join(ROOT, "distributed_gpu_test_amd", "_C.so")):
        assert fw["extension"] == os.path.join(img_home, "distributed_gpu_test_amd", "_C.so")


def test_sbatch_failure_propagates(tmp_path, image):
    r, sub, _ = _run_sbatch(tmp_path, image, "--epochs 1 --no-save --fail-at 0:end")
    assert r.returncode != 0
    assert (sub / "job_status.txt").read_text().strip() == "fail"
    assert "❌ job fail" in r.stdout


def test_sbatch_two_nodes(tmp_path, image):
    """2 nodes x 2 GPUs: one srun task per node runs torchrun --nnodes 2 --node-rank $SLURM_PROCID
    (reference slurm_train.sbatch:3-4,19-20,36); world size 4 gives the ws=4 oracle.  As in the
    reference (train.py:119-121) the local rank 0 of EACH node prints the average loss of its own
    shard: global rank 0 prints the oracle, global rank 2 (node 1) its own shard's value."""
    r, sub, _ = _run_sbatch(tmp_path, image, "--epochs 2", nodes=2, gpus=2)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert (sub / "job_status.txt").read_text().strip() == "success"
    assert r.stdout.count("Epoch  1 finished. Avg loss:") == 2
    assert r.stdout.count("Epoch  1 finished. Avg loss: 0.5857") >= 1
    assert r.stdout.count("Epoch  2 finished. Avg loss:") == 2
    assert r.stdout.count("Epoch  2 finished. Avg loss: 0.3375") >= 1
    assert r.stdout.count("Training completed.") == 2
    # one checkpoint tree in the shared submit dir, written by global rank 0 (node 0)
    assert (sub / "ds_checkpoints" / "epoch2" / "latest").exists()
    assert len(list((sub / "logs").glob("health_job*_node*.json"))) == 2


def test_sbatch_two_nodes_failure_on_node1(tmp_path, image):
    r, sub, _ = _run_sbatch(tmp_path, image, "--epochs 1 --no-save --fail-at 2:end", nodes=2, gpus=2)
    assert r.returncode != 0, r.stdout[-2000:]
    assert (sub / "job_status.txt").read_text().strip() == "fail"
    assert "❌ job fail" in r.stdout


@pytest.mark.parametrize("fail,want_rc", [(False, 0), (True, 1)])
def test_ci_submit_and_wait(tmp_path, image, fail, want_rc):
    sub = _submit_dir(tmp_path)
    env = _env(tmp_path, image, DGT_POLL_INTERVAL="1", DGT_POLL_MAX="240", DGT_STATUS_POLL_INTERVAL="1",
               FAKE_SLURM_GPUS="2", FAKE_SLURM_NODES="1",
               TRAIN_ARGS="--epochs 1 --no-save" + (" --fail-at 1:end" if fail else ""))
    r = subprocess.run(["bash", str(sub / "scripts" / "slurm_submit_and_wait.sh"), str(sub)],
                       cwd=sub, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == want_rc, r.stdout[-3000:] + r.stderr[-2000:]
    rendered = (sub / "slurm_train.submit.sbatch").read_text()
    assert "#SBATCH --nodes=1" in rendered and "#SBATCH --gres=gpu:2" in rendered
    assert "Submitted batch job" in r.stdout


def test_ci_submit_timeout_cancels(tmp_path, image):
    sub = _submit_dir(tmp_path)
    env = _env(tmp_path, image, DGT_POLL_INTERVAL="1", DGT_POLL_MAX="2", FAKE_SLURM_GPUS="2",
               TRAIN_ARGS="--epochs 1 --no-save --fail-at 0:1:hang")
    r = subprocess.run(["bash", str(sub / "scripts" / "slurm_submit_and_wait.sh"), str(sub)],
                       cwd=sub, env=env, capture_output=True, text=True, timeout=200)
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
