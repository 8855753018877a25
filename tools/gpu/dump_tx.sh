set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for w in crc32 qsort intmix hello fpamo; do
SHREWD_FI_DUMP_TX=gpurun_out/tx_$w.inc SHREWD_FI_NO_SOLO_TX=1 timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'.')
from shrewd_amd import Engine
e=Engine(); e.load_elf(open('workloads/$w.elf','rb').read(),['$w']); g=e.golden_run(); print('$w', g.translated_blocks, e.translate_status()[:200])
" || exit 1
done
