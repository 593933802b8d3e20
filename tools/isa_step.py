"""Issue position of the non-MFMA instructions of a kernel's k-step block, in MFMA slots.

  python tools/isa_step.py k.s <mangled-name-substring> [block-label]

Picks the basic block with the most MFMAs (or the given label) of the first kernel whose name
contains the substring, and prints each non-MFMA instruction prefixed by the number of MFMAs
issued before it -- e.g. where the global loads of the next k-step and their vmcnt wait land.
"""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    want = sys.argv[3] if len(sys.argv) > 3 else None
    s = open(path).read().split("\n")
    st = next(i for i, l in enumerate(s) if re.match(r"^_Z\S*:", l) and pat in l.split(":")[0])
    end = next(i for i in range(st, len(s)) if s[i].strip().startswith(".Lfunc_end"))
    blocks, cur, lab = [], [], "entry"
    for t in (x.strip() for x in s[st + 1:end]):
        m = re.match(r"^(\.LBB\d+_\d+):", t)
        if m:
            blocks.append((lab, cur))
            lab, cur = m.group(1), []
        elif t and not t.startswith(";") and not t.startswith("."):
            cur.append(t)
    blocks.append((lab, cur))
    if want:
        lab, ins = next(b for b in blocks if b[0] == want)
    else:
        lab, ins = max(blocks, key=lambda b: sum("mfma" in x for x in b[1]))
    print(s[st].split(":")[0], lab)
    mf = 0
    for t in ins:
        if "mfma" in t:
            mf += 1
            continue
        print(f"[{mf:2d}] {t[:100]}")


if __name__ == "__main__":
    main()
