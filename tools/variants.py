"""Score-kernel tuning variants (C2 instance only, -DKGE_ONLY_ONE).

    python tools/variants.py build NAME -DKGE_SLOTS_PER_WAVE=128 ...   # here: KGE/_lib/libkge_var_NAME.so
    python tools/variants.py buildfull NAME -D...   # every model family (all library sources)
    python tools/variants.py run NAME [NAME ...] [-- --workload c2-50m]  # on the GPU box: bench.py per variant
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "knowledge-graph-embedding_amd", "csrc")
LIBDIR = os.path.join(ROOT, "knowledge-graph-embedding_amd", "KGE", "_lib")


def build(name, defines, full=False):
    objs, procs = [], []
    if full:
        sys.path.insert(0, ROOT)
        import __graft_entry__
        sources, defines = __graft_entry__.SOURCES, list(defines)
    else:
        sources, defines = ("kge_step.hip", "kge_abi.hip", "kge_transr.hip", "kge_rel.hip", "kge_stream.hip", "kge_exchange.hip",
                            "kge_owner_transe.hip", "kge_owner_other.hip"), \
            ["-DKGE_ONLY_ONE"] + list(defines)
    for src in sources:
        # single-instance builds: the knobs are the score / update kernels' (kge_step.hip)
        # and the plan's (kge_abi.hip: KGE_STEP_WAVES, KGE_SLOTS_PER_WAVE size the launch);
        # the other units are compiled once, shared by every variant
        shared = not full and src not in ("kge_step.hip", "kge_abi.hip")
        obj = "/tmp/var_%s_%s" % ("shared" if shared else name, src.replace(".hip", ".o"))
        if shared and os.path.exists(obj):
            objs.append(obj)
            continue
        cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC"] + \
              (["-DKGE_ONLY_ONE"] if shared else defines) + ["-c", os.path.join(CSRC, src), "-o", obj]
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    for p in procs:
        assert p.wait() == 0
    out = os.path.join(LIBDIR, "libkge_var_%s.so" % name)
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", out], check=True)
    print("built", out)


def run(names, extra=()):
    import json
    for n in names:
        env = dict(os.environ, KGE_LIB=os.path.join(LIBDIR, "libkge_var_%s.so" % n))
        out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-hbm-point"]
                             + list(extra), env=env,
                             capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(n, "FAILED", out.stderr[-800:])
            continue
        d = json.loads(line[-1])
        k = (d.get("roofline") or {}).get("kernels") or {}
        ks, ku = (k.get("score_kernel") or {}).get("ms"), (k.get("update_kernel") or {}).get("ms")
        print("%-12s %.5f ms/step  KS %s  KU %s" % (n, d["ms_per_step"], ks, ku), flush=True)


if __name__ == "__main__":
    if sys.argv[1] in ("build", "buildfull"):
        build(sys.argv[2], sys.argv[3:], full=sys.argv[1] == "buildfull")
    else:   # run NAME [NAME ...] [-- bench.py arguments]
        a = sys.argv[2:]
        cut = a.index("--") if "--" in a else len(a)
        run(a[:cut], a[cut + 1:])
