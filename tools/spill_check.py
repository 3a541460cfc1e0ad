"""Register / scratch check of every prebuilt configuration's kernels (development).

Compiles each config's device code with -save-temps into a scratch directory and prints every
kernel that uses scratch (spills) plus the VGPR / AGPR counts of the whole-solve kernels, so a
change that pushes a kernel into spilling is seen before a GPU run.
Usage: python tools/spill_check.py [substring ...]   (default: all configs)."""
import importlib
import os
import re
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd")
from ude_amd import _native, configs  # noqa: E402

pats = sys.argv[1:]
sel = [(i, c) for i, c in enumerate(configs.PREBUILT) if not pats or any(p in configs.config_key(c) for p in pats)]
gen = os.path.join(_native.BUILD, "gen_prebuilt")
tmp = tempfile.mkdtemp(prefix="ude_spill_")


def one(ic):
    i, c = ic
    d = os.path.join(tmp, str(i))
    os.makedirs(d)
    cmd = [_native.HIPCC, *_native.HIP_FLAGS, *os.environ.get("SPILL_FLAGS", "").split(), "--offload-device-only", "-S", "-I", _native.INCLUDE, "-I",
           _native.CSRC, "-I", gen, os.path.join(_native.CSRC, "ude_cfg.hip"), f"-DUDE_CFG_ID={i}",
           f"-DUDE_ONE_CONFIG={configs.template_args(c)}", "-o", os.path.join(d, "k.s")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return configs.config_key(c), None, r.stderr[-2000:]
    return configs.config_key(c), open(os.path.join(d, "k.s")).read(), ""


def scratch_ops(txt):
    """scratch load / store instructions per kernel symbol (a private segment without any is an
    unused private array, not a spill)"""
    ops, cur = {}, None
    for ln in txt.split("\n"):
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            cur = m.group(1)
        elif cur and "scratch_" in ln and not ln.lstrip().startswith(";"):
            ops[cur] = ops.get(cur, 0) + 1
    return ops


bad = 0
with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
    for key, txt, err in ex.map(one, sel):
        if txt is None:
            print(f"{key}: BUILD FAILED\n{err}")
            bad += 1
            continue
        ops = scratch_ops(txt)
        for blk in re.findall(r"\n\s+- \.agpr_count:.*?(?=\n\s+- \.agpr_count:|\n\.end_amdgpu_metadata)", txt, re.S):
            f = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
            name = f.get("name", "?")
            scratch = int(f.get("private_segment_fixed_size", "0"))
            short = re.sub(r"ude::Model<[^>]*>", "M", subprocess.run(["c++filt"], input=name, capture_output=True,
                                                                     text=True).stdout.strip())[:90]
            nops = ops.get(name, 0)
            if scratch > 0 and nops > 0:
                bad += 1
                print(f"SPILL {key:34s} scratch {scratch:5d} B {nops:4d} ops vgpr {f.get('vgpr_count')} {short}")
            elif "ude_bwd_kernel" in name or "ude_fwd_kernel" in name:
                print(f"      {key:34s} vgpr {f.get('vgpr_count'):>4} agpr {f.get('agpr_count'):>4} {short}")
print("spilling kernels / failed builds:", bad)
sys.exit(1 if bad else 0)
