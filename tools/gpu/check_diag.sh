# GPU parity tests, the default bench line, and the slow-seed diagnostic
set -o pipefail
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
python -c "import json;b=json.load(open('gpurun_out/bench.json'));print('bench', round(b['value']), b['ms_per_step'], b['outcomes'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --seed 0x5EED0003 > gpurun_out/bench3.json 2> gpurun_out/bench3.err || exit 1
python -c "import json;b=json.load(open('gpurun_out/bench3.json'));print('bench seed3', round(b['value']), b['ms_per_step'], b['outcomes'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload qsort --steps 2 > gpurun_out/benchq.json 2> gpurun_out/benchq.err || exit 1
python -c "import json;b=json.load(open('gpurun_out/benchq.json'));print('bench qsort', round(b['value']), b['ms_per_step'], b['outcomes'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload intmix --steps 1 > gpurun_out/benchi.json 2> gpurun_out/benchi.err || exit 1
python -c "import json;b=json.load(open('gpurun_out/benchi.json'));print('bench intmix', round(b['value']), b['ms_per_step'], b['outcomes'])"
