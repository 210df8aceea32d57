#!/bin/bash
# CI "test-on-slurm" step as a script (testable against tests/fake_slurm): size the job to the
# cluster, submit slurm_train.sbatch, wait for it to leave the queue, then turn the job's
# job_status.txt into this script's exit code.  Same contract as the reference's inline CI step
# (.github/workflows/distributed-gpu-test-ci.yaml:107-181 there).
#
#   scripts/slurm_submit_and_wait.sh [SUBMIT_DIR]
#
# Sizing: nodes = NodeName lines of `scontrol show nodes` (DGT_NODES overrides), GPUs per node =
# gres/gpu of the first node's CfgTRES (DGT_GPUS_PER_NODE overrides; 8 if none is reported).
# Exit codes: 0 success | 1 job failed, or status unknown / missing | 2 sbatch failed |
# 124 the job was still queued/running at the deadline (it is cancelled).
# Timing knobs: DGT_POLL_INTERVAL (10 s) x DGT_POLL_MAX (30) for the queue,
# DGT_STATUS_POLL_INTERVAL (10 s) x DGT_STATUS_POLL_MAX (3) for the status file.
set -euo pipefail

SUBMIT_DIR=${1:-$PWD}
cd "$SUBMIT_DIR"
STATUS_FILE="$PWD/job_status.txt"

log() { echo "[submit] $*"; }

cluster_shape() {
  local nodes_out
  nodes_out=$(scontrol show nodes)
  N_NODES=${DGT_NODES:-$(grep -c '^NodeName' <<<"$nodes_out" || true)}
  N_GPUS=${DGT_GPUS_PER_NODE:-$(grep -o 'gres/gpu=[0-9]*' <<<"$nodes_out" | head -n 1 | cut -d= -f2 || true)}
  [ "${N_NODES:-0}" -ge 1 ] 2>/dev/null || N_NODES=1
  [ "${N_GPUS:-0}" -ge 1 ] 2>/dev/null || N_GPUS=8
}

render_job() {  # the sbatch with its #SBATCH geometry rewritten for this cluster
  awk -v n="$N_NODES" -v g="$N_GPUS" '
    /^#SBATCH --nodes=/   { print "#SBATCH --nodes=" n; next }
    /^#SBATCH --gres=gpu:/ { print "#SBATCH --gres=gpu:" g; next }
    { print }' slurm_train.sbatch > slurm_train.submit.sbatch
}

submit() {
  local out
  out=$(sbatch --export=ALL,GPUS_PER_NODE="$N_GPUS",NNODES="$N_NODES" slurm_train.submit.sbatch || true)
  JOB_ID=$(awk '/Submitted batch job/ { print $NF }' <<<"$out")
  if [ -z "$JOB_ID" ]; then
    log "sbatch did not return a job id; output: '$out'"
    exit 2
  fi
  log "Submitted batch job $JOB_ID (nodes=$N_NODES gpus/node=$N_GPUS)"
}

wait_for_queue_exit() {
  local every=${DGT_POLL_INTERVAL:-10} max=${DGT_POLL_MAX:-30} n state
  for (( n = 1; n <= max; n++ )); do
    state=$(squeue -j "$JOB_ID" -h -o "%T" 2>/dev/null | tr -d '\r' || true)
    if [ -z "$state" ]; then
      log "job $JOB_ID left the queue after $n check(s)"
      return 0
    fi
    log "job $JOB_ID is $state; next check in ${every}s"
    sleep "$every"
  done
  log "job $JOB_ID still queued/running after $((every * max))s: cancelling it"
  scancel "$JOB_ID" || true
  exit 124
}

verdict() {
  local every=${DGT_STATUS_POLL_INTERVAL:-10} max=${DGT_STATUS_POLL_MAX:-3} n status
  for (( n = 1; n <= max; n++ )); do
    if [ -f "$STATUS_FILE" ]; then
      status=$(tr -d '\r\n' < "$STATUS_FILE" || true)
      log "$STATUS_FILE says '$status'"
      case "$status" in
        success|0) exit 0 ;;
        fail|1) log "the job reported failure"; exit 1 ;;
        *) log "unrecognised status '$status': failing"; exit 1 ;;
      esac
    fi
    log "no $STATUS_FILE yet (shared filesystem lag?); next check in ${every}s"
    sleep "$every"
  done
  log "$STATUS_FILE never appeared: failing"
  exit 1
}

cluster_shape
render_job
rm -f "$STATUS_FILE"
submit
wait_for_queue_exit
verdict
