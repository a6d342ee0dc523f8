"""Per-kernel register / spill / LDS summary from a hipcc --cuda-device-only -S listing.
usage: python tools/kernel_regs.py file.s [name-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
sub = sys.argv[2] if len(sys.argv) > 2 else ""
meta = s[s.index("amdhsa.kernels:"):]
for ent in re.split(r"\n\s+- \.agpr_count:", meta)[1:]:
    def f(k):
        m = re.search(r"\.%s:\s+(\S+)" % k, ent)
        return m.group(1) if m else "?"
    name = f("name")
    if sub not in name:
        continue
    agpr = ent.split("\n", 1)[0].strip()
    print(f"{name[:90]:90s} vgpr={f('vgpr_count'):>4s} agpr={agpr:>4s} sgpr={f('sgpr_count'):>4s} "
          f"vspill={f('vgpr_spill_count')} sspill={f('sgpr_spill_count')} lds={f('group_segment_fixed_size')} "
          f"priv={f('private_segment_fixed_size')}")
