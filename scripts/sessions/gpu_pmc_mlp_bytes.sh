set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --model mlp --steps 5 --warmup 2 > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --model mlp --steps 5 --warmup 2 > gpurun_out/pmc_write.log 2>&1 && echo ok
