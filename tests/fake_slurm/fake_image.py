"""Build a FAKE container image directory from the repository's Dockerfile (for tests/fake_slurm/srun).

Only what the job can observe is emulated: the image's ENV and WORKDIR, the files its COPY lines
place (honouring .dockerignore), and the outputs of the ``tools/build_ext.py`` RUN step (the
in-tree ``_C.so`` and ``build/bin`` tools, copied to where that RUN step would have written them).
The result is ``<dst>/.fake_image.json`` + the image's files under ``<dst>/<absolute path>``.
"""
from __future__ import annotations

import fnmatch
import json
import os
import re
import shlex
import shutil
from typing import Dict, List

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _logical_lines(text: str) -> List[str]:
    out, cur = [], ""
    for raw in text.splitlines():
        line = raw.rstrip()
        if not cur and (not line.strip() or line.lstrip().startswith("#")):
            continue
        if line.endswith("\\"):
            cur += line[:-1] + " "
            continue
        out.append((cur + line).strip())
        cur = ""
    if cur:
        out.append(cur.strip())
    return out


def _ignore_patterns(root: str) -> List[str]:
    p = os.path.join(root, ".dockerignore")
    if not os.path.exists(p):
        return []
    return [l.strip() for l in open(p) if l.strip() and not l.startswith("#")]


def _ignored(rel: str, pats: List[str]) -> bool:
    rel = rel.replace(os.sep, "/")
    for pat in pats:
        pat = pat.rstrip("/")
        cands = [pat] + ([pat[3:]] if pat.startswith("**/") else [])
        for c in cands:
            if fnmatch.fnmatch(rel, c) or any(fnmatch.fnmatch(rel, c + "/*") for _ in [0]):
                return True
            if "/" not in c and any(fnmatch.fnmatch(part, c) for part in rel.split("/")):
                return True
    return False


def _copy(src_rel: str, dst_abs: str, img: str, pats: List[str], root: str) -> None:
    src = os.path.join(root, src_rel)
    target = os.path.join(img, dst_abs.lstrip("/"))
    if os.path.isdir(src):
        for dp, dns, fns in os.walk(src):
            rel_dir = os.path.relpath(dp, root)
            dns[:] = [d for d in dns if not _ignored(os.path.join(rel_dir, d), pats)]
            for f in fns:
                rel = os.path.normpath(os.path.join(rel_dir, f))
                if _ignored(rel, pats):
                    continue
                out = os.path.join(target, os.path.relpath(os.path.join(dp, f), src))
                os.makedirs(os.path.dirname(out), exist_ok=True)
                shutil.copy2(os.path.join(dp, f), out)
    else:
        if dst_abs.endswith("/"):
            target = os.path.join(target, os.path.basename(src_rel))
        os.makedirs(os.path.dirname(target), exist_ok=True)
        shutil.copy2(src, target)


def build_fake_image(dst: str, root: str = ROOT, dockerfile: str = "Dockerfile") -> Dict:
    os.makedirs(dst, exist_ok=True)
    pats = _ignore_patterns(root)
    env: Dict[str, str] = {}
    workdir = "/"
    roots: List[str] = []
    for line in _logical_lines(open(os.path.join(root, dockerfile)).read()):
        instr, _, rest = line.partition(" ")
        instr = instr.upper()
        if instr == "ENV":
            for tok in shlex.split(rest):
                if "=" in tok:
                    k, v = tok.split("=", 1)
                    env[k] = v
        elif instr == "WORKDIR":
            workdir = rest.strip()
            os.makedirs(os.path.join(dst, workdir.lstrip("/")), exist_ok=True)
            roots.append(workdir)
        elif instr == "COPY":
            toks = [t for t in shlex.split(rest) if not t.startswith("--")]
            *srcs, d = toks
            if not d.startswith("/"):
                d = os.path.join(workdir, d)
            for s in srcs:
                _copy(s, d, dst, pats, root)
            roots.append(d.rstrip("/") if d.endswith("/") or len(srcs) > 1 else os.path.dirname(d))
        elif instr == "RUN" and "tools/build_ext.py" in rest:
            # (``cd DIR && ... && python3 tools/build_ext.py``: other commands may come between)
            m = re.search(r"cd\s+(\S+)\s*&&.*?python3?\s+tools/build_ext\.py", rest)
            where = m.group(1) if m else workdir
            so = os.path.join(root, "distributed_gpu_test_amd", "_C.so")
            if os.path.exists(so):
                out = os.path.join(dst, where.lstrip("/"), "distributed_gpu_test_amd", "_C.so")
                os.makedirs(os.path.dirname(out), exist_ok=True)
                shutil.copy2(so, out)
            bin_dir = os.path.join(root, "build", "bin")
            if os.path.isdir(bin_dir):
                shutil.copytree(bin_dir, os.path.join(dst, where.lstrip("/"), "build", "bin"), dirs_exist_ok=True)
    meta = {"env": env, "workdir": workdir, "roots": sorted(set(roots))}
    json.dump(meta, open(os.path.join(dst, ".fake_image.json"), "w"), indent=1)
    return meta


def ci_scp_files(root: str = ROOT) -> List[str]:
    """The file list the CI's scp step copies to the SLURM host (the job's submit directory)."""
    import yaml
    wf = yaml.safe_load(open(os.path.join(root, ".github", "workflows", "distributed-gpu-test-ci.yaml")))
    for step in wf["jobs"]["build"]["steps"]:
        if "scp-action" in str(step.get("uses", "")):
            return [s.strip() for s in step["with"]["source"].split(",") if s.strip()]
    raise RuntimeError("no scp step in the CI workflow")


def stage_submit_dir(dst: str, root: str = ROOT) -> List[str]:
    """A submit directory shaped like the CI's: ONLY the scp'd files (+ the .sqsh, faked separately)."""
    files = ci_scp_files(root)
    for f in files:
        out = os.path.join(dst, f)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        shutil.copy2(os.path.join(root, f), out)
    return files
