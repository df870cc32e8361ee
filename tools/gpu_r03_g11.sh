set -o pipefail
cd $GRAFT_REPO_ROOT
for w in 5 100 5 100; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup $w > gpurun_out/bench_w$w.json 2> gpurun_out/bench_w$w.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/bench_w$w.json')); print('warmup', $w, d['kernel_ms_avg'], d['ms_per_step'], d['roofline']['frac'])"
done
