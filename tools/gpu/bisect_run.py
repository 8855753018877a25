import json, sys, os
sys.path.insert(0, os.getcwd())
from shrewd_amd import Engine
exp = json.load(open('_dbg/exp.json'))
for k in sorted(exp, key=int):
    e = Engine()
    e.load_elf(open(f'_dbg/v{k}.elf', 'rb').read(), ['fpamo'])
    g = e.golden_run()
    out = e.golden_stdout().decode()
    ok = out == exp[k][0] and g.ninst == exp[k][1] and g.ncycles == exp[k][2]
    print(k, 'OK' if ok else 'DIFF', exp[k][3], out.strip(), exp[k][0].strip(), g.ninst, exp[k][1], g.ncycles, exp[k][2], flush=True)
    e.close()
    if not ok:
        break
