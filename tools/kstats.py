"""Per-kernel register / scratch / LDS summary of a gfx950 .s file (hipcc -save-temps)."""
import re
import subprocess
import sys

txt = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.findall(r"\n\s+- \.agpr_count:.*?(?=\n\s+- \.agpr_count:|\n\.end_amdgpu_metadata)", txt, re.S):
    f = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
    name = f.get("name", "?")
    if pat not in name:
        continue
    try:
        dm = subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
    except Exception:
        dm = name
    dm = re.sub(r"ude::Model<([^>]*)>", "M", dm)
    print(f"vgpr {f.get('vgpr_count'):>4} agpr {f.get('agpr_count'):>4} sgpr {f.get('sgpr_count'):>4} "
          f"scratch {f.get('private_segment_fixed_size'):>5}  {dm[:110]}")
