"""Per-basic-block instruction mix of kernels in a gfx950 assembly listing.

  hipcc -O3 --offload-arch=gfx950 -std=c++17 -Isparsergps_amd/csrc --cuda-device-only -S \
        -o /tmp/k.s sparsergps_amd/csrc/k_mfma.hip
  python tools/isa_blocks.py /tmp/k.s k_syrk_blk [min_mfma]

Prints, for every kernel whose mangled name contains the pattern, its VGPR / spill counts and
the blocks holding at least `min_mfma` MFMAs (default 1): instruction count and mix (MFMA, LDS
reads / writes, global loads, waitcnts, other VALU / SALU).
"""
import collections
import re
import sys


def kinds(ins):
    c = collections.Counter()
    for i in ins:
        if "mfma" in i:
            k = "mfma"
        elif i.startswith("ds_read"):
            k = "ds_read"
        elif i.startswith("ds_write"):
            k = "ds_write"
        elif i.startswith("global_load") or i.startswith("buffer_load"):
            k = "gload"
        elif i.startswith("s_waitcnt"):
            k = "waitcnt"
        elif i.startswith("v_"):
            k = "valu"
        elif i.startswith("s_"):
            k = "salu"
        else:
            k = "other"
        c[k] += 1
    return dict(c)


def main():
    path, pat = sys.argv[1], sys.argv[2]
    min_mfma = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    lines = open(path).read().split("\n")
    meta = {}
    cur = None
    for ln in lines:   # amdhsa metadata: .name then counts, per kernel
        t = ln.strip()
        m = re.match(r"\.name:\s+(\S+)", t)
        if m:
            cur = m.group(1)
            meta.setdefault(cur, {})
        m = re.match(r"\.(vgpr_count|vgpr_spill_count|agpr_count):\s+(\d+)", t)
        if m and cur:
            meta[cur][m.group(1)] = int(m.group(2))
    for idx, ln in enumerate(lines):
        m = re.match(r"^(_Z\S+):", ln)
        if not m or pat not in m.group(1):
            continue
        name = m.group(1)
        end = next(i for i in range(idx, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
        blocks, ins, lab = [], [], "entry"
        for t in (x.strip() for x in lines[idx + 1:end]):
            lm = re.match(r"^(\.LBB\d+_\d+):", t)
            if lm:
                blocks.append((lab, ins))
                lab, ins = lm.group(1), []
            elif t and not t.startswith(";") and not t.startswith("."):
                ins.append(t.split()[0])
        blocks.append((lab, ins))
        print(name, meta.get(name, {}))
        for lab, ins in blocks:
            k = kinds(ins)
            if k.get("mfma", 0) >= min_mfma:
                print("   ", lab, len(ins), k)


if __name__ == "__main__":
    main()
