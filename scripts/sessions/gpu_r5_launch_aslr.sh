# round 5: the one-node graph replay costs ~2.6 us of host time in some fresh processes and ~10 us in
# others (gpu_r5_launch_var.sh).  Is it the address-space layout?  Eight probe processes with address
# randomisation off (setarch -R: the personality flag is set before python starts, nothing touches
# the GPU before the exec) and eight with it on, alternating.
set -o pipefail
O=${OUT:-gpurun_out/r5la}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 120 setarch "$(uname -m)" -R python scripts/graph_launch_probe.py > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
  grep launch-probe $O/p.log | sed 's/^/norand /' | tee -a $O/aslr.txt
  timeout -k 10 120 python scripts/graph_launch_probe.py > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
  grep launch-probe $O/p.log | sed 's/^/rand   /' | tee -a $O/aslr.txt
done
echo done
