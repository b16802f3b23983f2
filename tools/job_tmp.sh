set -o pipefail
mkdir -p gpurun_out/j27
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/j27/bench.json 2> gpurun_out/j27/bench.err && \
timeout -k 10 600 python bench.py --no-cpu-baseline --no-kernel-timing > gpurun_out/j27/bench_nt.json 2>> gpurun_out/j27/bench.err
python3 -c "
import json
for f in ['gpurun_out/j27/bench.json','gpurun_out/j27/bench_nt.json']:
    d=json.load(open(f)); print(f, d['ms_per_step'], d['value'], json.dumps(d['roofline'])); print({k:(round(v['ms']*1e3,1), round(v['ms_isolated']*1e3,1), v['launches_timed']) for k,v in d['kernels'].items()})
"
