set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ep_sweep_r05${TAG}.jsonl
for wl in "crc32:" "qsort:--workload qsort" "intmix:--workload intmix --trials 125000"; do
  name=${wl%%:*}; args=${wl#*:}
  for ei in ${EIS:-1024 512 2048 4096}; do
    timeout -k 10 300 python -u bench.py --workloads "" --no-cpu-baseline --steps 6 --epoch-iters $ei $args > gpurun_out/ep_one.json 2> gpurun_out/ep_one.err || exit $?
    python - "$name" "$ei" >> gpurun_out/ep_sweep_r05${TAG}.jsonl <<'PY'
import json, sys
d = json.load(open("gpurun_out/ep_one.json"))
print(json.dumps({"workload": sys.argv[1], "epoch_iters": int(sys.argv[2]), "ms_per_step": round(d["ms_per_step"], 4), "value": round(d["value"])}))
PY
    tail -n 1 gpurun_out/ep_sweep_r05${TAG}.jsonl
  done
done
