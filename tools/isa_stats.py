#!/usr/bin/env python3
"""Instruction mix and register budget of the gfx950 kernels in a hipcc
object (``csrc/build/*.o``): extracts the offload bundle, disassembles it and
prints, per kernel matching a substring, the static count of each
instruction class plus the VGPR / AGPR / SGPR / LDS / scratch figures of the
code-object notes.

    python tools/isa_stats.py ska-sdp-screen-fitting_amd/csrc/build/kl_eval.o \
        'kl_eval_kernelILi13ELi4ELb1ELb1ELb1ELb0ELb1E' [--dump]
"""
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    obj, pat = sys.argv[1], sys.argv[2]
    dump = "--dump" in sys.argv
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        co = os.path.join(d, "k.co")
        subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", obj], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        f"--input={fat}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--output={co}"], check=True)
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True,
                             capture_output=True, text=True).stdout
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    blocks = re.split(r"\n(?=[0-9a-f]+ <)", dis)
    for b in blocks:
        m = re.match(r"[0-9a-f]+ <(\S+)>:", b)
        if not m or pat not in m.group(1) or m.group(1).endswith(".kd"):
            continue
        name = m.group(1)
        ins = [ln.split()[0] for ln in b.splitlines()[1:] if ln.strip() and not ln.strip().startswith(";")
               and re.match(r"\s+\S", ln)]
        c = Counter()
        for i in ins:
            if i.startswith("v_mfma"):
                c["mfma"] += 1
            elif i.startswith(("global_store", "buffer_store")):
                c["vmem_store"] += 1
            elif i.startswith(("global_load", "buffer_load")):
                c["vmem_load"] += 1
            elif i.startswith("ds_"):
                c["lds"] += 1
            elif i.startswith(("s_", )):
                c["salu/smem/ctrl"] += 1
            elif i.startswith(("v_sin", "v_cos", "v_exp", "v_log", "v_rcp", "v_sqrt", "v_rsq")):
                c["valu_trans"] += 1
            elif re.match(r"v_\w+_f64", i):
                c["valu_f64"] += 1
            elif i.startswith("v_accvgpr"):
                c["accvgpr_copy"] += 1
            elif i.startswith("scratch_"):
                c["scratch"] += 1
            elif i.startswith("v_"):
                c["valu_other"] += 1
            else:
                c["other:" + i] += 1
        meta = {}
        i = notes.find(".name:           " + name)
        if i < 0:
            i = notes.find(name)
        seg = notes[max(0, i - 3000):i + 400]
        for k in (".vgpr_count", ".agpr_count", ".sgpr_count", ".group_segment_fixed_size",
                  ".private_segment_fixed_size", ".vgpr_spill_count"):
            mm = re.findall(re.escape(k) + r":\s+(\d+)", seg)
            if mm:
                meta[k[1:]] = int(mm[-1])
        print(name)
        print("  ", meta)
        print("  ", dict(sorted(c.items())), "total", len(ins))
        if dump:
            print(b)


if __name__ == "__main__":
    main()
