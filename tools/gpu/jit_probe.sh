#!/bin/bash
# Load-time build probe: golden run of each workload with JIT tracing, each in
# its own process (run via gpurun).
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache_probe SHREWD_FI_TRACE=1
for w in ${@:-crc32 qsort}; do
timeout -k 10 120 python -X faulthandler -c "
import sys; sys.path.insert(0,'.')
from shrewd_amd import Engine
e=Engine(); e.load_elf(open('workloads/$w.elf','rb').read(),['$w']); g=e.golden_run(); print('$w', g.translated_blocks, repr(e.translate_status()[:300]), flush=True)
e.set_campaign(5, (1<<33)-2, 1); o,h=e.run_trials(0, 3000); print('$w trials ok', h['trials'], flush=True)
" > gpurun_out/jit_probe_$w.log 2>&1; echo "$w rc=$?"; grep -v "^  File\|^Extension\|^Thread\|^Current\|^$" gpurun_out/jit_probe_$w.log | tail -8
done
