"""Print per-kernel VGPR / AGPR / spill / LDS usage from a hipcc -save-temps .s file (amdhsa metadata)."""
import re
import sys

txt = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.split(r"\n\s+- \.", txt.split("amdhsa.kernels:")[1]):
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or pat not in name.group(1):
        continue
    get = lambda k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "?"])[1]
    print(f"vgpr={get('vgpr_count'):>4} agpr={get('agpr_count'):>4} vspill={get('vgpr_spill_count'):>4} "
          f"lds={get('group_segment_fixed_size'):>6} {name.group(1)[:110]}")
