set -o pipefail
timeout -k 10 240 python bench.py --workload gossip --no-cpu-baseline > gpurun_out/g_dense.log 2>&1 && \
timeout -k 10 240 python bench.py --workload gossip --engine sparse --no-cpu-baseline > gpurun_out/g_sparse.log 2>&1 && \
timeout -k 10 240 python bench.py --jitter --no-cpu-baseline > gpurun_out/pj.log 2>&1
for f in g_dense g_sparse pj; do echo "== $f"; tail -1 gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_us'], d['roofline']['frac'])" || tail -5 gpurun_out/$f.log; done
