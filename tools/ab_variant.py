"""Builds an A/B variant of the engine library from a patched copy of the
sources (never the tree itself): python tools/ab_variant.py NAME 'OLD=>NEW' ...
Each argument replaces one exact, unique text of shrewd_amd/csrc/hip/
fi_trial.hip (or FILE::OLD=>NEW for another file under shrewd_amd/csrc).  The
library and its own JIT helper (which embeds the patched kernel source) go to
shrewd_amd/_lib/NAME/, for tools/gpu/ab_bench.sh NAME/libshrewd_fi.so."""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    name, patches = sys.argv[1], sys.argv[2:]
    work = os.path.join("/tmp", "ab_variant", name)
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    shutil.copytree(os.path.join(ROOT, "shrewd_amd"), os.path.join(work, "shrewd_amd"),
                    ignore=shutil.ignore_patterns("_lib", "__pycache__"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(work, "include"))
    for p in patches:
        fname, _, rest = p.rpartition("::")
        path = os.path.join(work, "shrewd_amd", "csrc", fname or os.path.join("hip", "fi_trial.hip"))
        old, new = rest.split("=>", 1)
        text = open(path).read()
        assert text.count(old) == 1, (p, text.count(old))
        open(path, "w").write(text.replace(old, new))
    out = os.path.join(ROOT, "shrewd_amd", "_lib", name)
    os.makedirs(out, exist_ok=True)
    sys.path.insert(0, work)
    import shrewd_amd.build as b   # the copy's build.py: paths inside `work`
    assert b.ROOT.startswith(work), b.ROOT
    b.build(force=True, out=os.path.join(out, "libshrewd_fi.so"))
    jitc = b.build_jitc(force=True)
    shutil.copy2(jitc, os.path.join(out, "fi_jitc"))
    print(out)


if __name__ == "__main__":
    main()
