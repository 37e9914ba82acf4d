cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cm -o cm -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_cm.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o cm -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o cm -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_write.log 2>&1
