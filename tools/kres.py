#!/usr/bin/env python3
"""Resource usage (LDS, VGPRs, SGPRs, spills, scratch) of the gfx950 kernels in a hipcc object:
python3 tools/kres.py pktvisor_amd/build/pv_kernels.o 'pv_topn_(merge|combine)$'"""
import os, re, subprocess, sys, tempfile

LLVM = "/opt/rocm/lib/llvm/bin/"
obj, pat = sys.argv[1], re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
with tempfile.TemporaryDirectory() as t:
    subprocess.check_call([LLVM + "llvm-objcopy", f"--dump-section=.hip_fatbin={t}/fat.bin", obj, f"{t}/o"])
    subprocess.check_call([LLVM + "clang-offload-bundler", "--unbundle", "--type=o", f"--input={t}/fat.bin",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={t}/k.co"])
    txt = subprocess.check_output([LLVM + "llvm-readelf", "--notes", f"{t}/k.co"], text=True)
for blk in txt.split("  - .agpr_count")[1:]:
    m = re.search(r"\.name:\s+(\S+)", blk)
    if not m or not pat.search(m.group(1)):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    print(f"{m.group(1):28s} lds={g('group_segment_fixed_size')} vgpr={g('vgpr_count')} sgpr={g('sgpr_count')} "
          f"vspill={g('vgpr_spill_count')} scratch={g('private_segment_fixed_size')} maxwg={g('max_flat_workgroup_size')}")
