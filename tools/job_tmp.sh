set -o pipefail
mkdir -p gpurun_out/j12
timeout -k 10 600 python bench.py > gpurun_out/j12/bench.json 2> gpurun_out/j12/bench.err && cat gpurun_out/j12/bench.json
