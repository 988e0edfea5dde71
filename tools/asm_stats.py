#!/usr/bin/env python3
"""Per-kernel instruction counts from a device assembly listing.

  hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=on --cuda-device-only -S \
      -o build/k.s differentiable-ilqr_amd/csrc/dilqr_kernels.hip
  python tools/asm_stats.py build/k.s [substring ...]

Static counts (not executed counts) of the instruction classes that matter for
the hot kernels, plus the compiler's VGPR / scratch figures.
"""
import re
import sys

CLASSES = {
    "valu": r"\tv_(?!mfma)",
    "pk_fma": r"\tv_pk_fma_f32",
    "fma": r"\tv_fmac?_f32",
    "dpp": r"row_mirror|row_half_mirror|quad_perm|row_sh|row_ror",
    "bpermute": r"\tds_bpermute",
    "ds_read": r"\tds_read",
    "ds_write": r"\tds_write",
    "gload": r"\tglobal_load",
    "gstore": r"\tglobal_store",
    "waitcnt_vm0": r"s_waitcnt vmcnt\(0\)",
    "barrier": r"\ts_barrier",
}


def main(path, subs):
    s = open(path).read()
    starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\S+):\s*;\s*@", s, re.M)]
    for i, (pos, name) in enumerate(starts):
        end = starts[i + 1][0] if i + 1 < len(starts) else len(s)
        body = s[pos:end]
        if subs and not any(x in name for x in subs):
            continue
        meta = s[end:end + 4000] if i + 1 == len(starts) else body
        vg = re.findall(r"\.vgpr_count:\s*(\d+)|NumVgprs:\s*(\d+)", s[pos:end + 20000])
        sc = re.findall(r"ScratchSize:\s*(\d+)", s[pos:end + 20000])
        counts = {k: len(re.findall(p, body)) for k, p in CLASSES.items()}
        vgpr = next((a or b for a, b in vg), "?")
        print(f"{name[:90]}\n   " + " ".join(f"{k}={v}" for k, v in counts.items())
              + f" vgpr={vgpr} scratch={sc[0] if sc else '?'}")
        del meta


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
