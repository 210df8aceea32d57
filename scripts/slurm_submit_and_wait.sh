#!/bin/bash
# Submit slurm_train.sbatch on a SLURM login node and wait for its verdict (the CI's
# "test-on-slurm" step, reference .github/workflows/distributed-gpu-test-ci.yaml:107-181, moved
# into a script so it can be tested against fake SLURM commands).
#
#   scripts/slurm_submit_and_wait.sh [REMOTE_DIR]
#
# Cluster discovery: NODES = number of nodes (DGT_NODES overrides; the reference counts every
# node of the cluster), GPUS = gres/gpu of the first node's CfgTRES (DGT_GPUS_PER_NODE overrides).
# Exit codes (same as the reference): 0 success, 1 fail / unknown / missing status,
# 2 submission failed, 124 job did not leave squeue in time.
set -euo pipefail

REMOTE_DIR=${1:-$PWD}
cd "$REMOTE_DIR"

NODES=${DGT_NODES:-$(scontrol show nodes | grep -c '^NodeName')}
GPUS=${DGT_GPUS_PER_NODE:-$(scontrol show nodes | sed -n 's/.*CfgTRES=.*gres\/gpu=\([0-9][0-9]*\).*/\1/p' | head -n1)}
GPUS=${GPUS:-8}
sed -e "s/^#SBATCH --nodes=.*/#SBATCH --nodes=${NODES}/" \
    -e "s/^#SBATCH --gres=gpu:.*/#SBATCH --gres=gpu:${GPUS}/" \
    slurm_train.sbatch > slurm_train.submit.sbatch
rm -f "$PWD/job_status.txt"
SBATCH_OUT=$(sbatch --export=ALL,GPUS_PER_NODE="$GPUS",NNODES="$NODES" slurm_train.submit.sbatch || true)
if [ -z "$SBATCH_OUT" ]; then
  echo "Failed to submit job; sbatch output: $SBATCH_OUT"
  exit 2
fi
JOB_ID=$(echo "$SBATCH_OUT" | awk '{print $NF}')
echo "Submitted batch job $JOB_ID (nodes=$NODES gpus/node=$GPUS)"

JOB_POLL_INTERVAL=${DGT_POLL_INTERVAL:-10}
JOB_POLL_MAX=${DGT_POLL_MAX:-30}
STATE=""
for (( i=0; i<JOB_POLL_MAX; i++ )); do
  STATE=$(squeue -j "$JOB_ID" -h -o "%T" 2>/dev/null | tr -d '\r' || true)
  if [ -z "$STATE" ]; then
    echo "Job $JOB_ID no longer in squeue (checked $((i+1)) times)"
    break
  fi
  echo "Job $JOB_ID state: $STATE — sleeping ${JOB_POLL_INTERVAL}s..."
  sleep "$JOB_POLL_INTERVAL"
done
if [ -n "$STATE" ]; then
  echo "Job $JOB_ID still in squeue after $((JOB_POLL_MAX * JOB_POLL_INTERVAL)) seconds; cancelling."
  scancel "$JOB_ID" || true
  exit 124
fi

STATUS_FILE="$PWD/job_status.txt"
STATUS_POLL_INTERVAL=${DGT_STATUS_POLL_INTERVAL:-10}
STATUS_POLL_MAX=${DGT_STATUS_POLL_MAX:-3}
for (( j=0; j<STATUS_POLL_MAX; j++ )); do
  if [ -f "$STATUS_FILE" ]; then
    STATUS=$(tr -d '\r' < "$STATUS_FILE" || true)
    echo "Found $STATUS_FILE -> '$STATUS'"
    case "$STATUS" in
      success|0) exit 0 ;;
      fail|1) echo "Remote job reported fail"; exit 1 ;;
      *) echo "Unknown status file content: '$STATUS' — treating as failure"; exit 1 ;;
    esac
  fi
  echo "Status file not present yet — sleeping ${STATUS_POLL_INTERVAL}s..."
  sleep "$STATUS_POLL_INTERVAL"
done
echo "$STATUS_FILE did not appear after $((STATUS_POLL_MAX * STATUS_POLL_INTERVAL)) seconds — treating as failure"
exit 1
