"""Instruction histogram of one kernel in a hipcc -S (device) listing.

    python tools/isa_hist.py <file.s> <symbol-substring> [top]
"""
import collections
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    s = open(path).read()
    m = re.search(r"^(\S*" + re.escape(pat) + r"\S*):", s, re.M)
    if not m:
        print("symbol not found")
        return 1
    i = m.start()
    j = s.index(".Lfunc_end", i)
    c = collections.Counter()
    for line in s[i:j].splitlines():
        t = line.strip().split()
        if t and not t[0].startswith((".", ";")) and not t[0].endswith(":"):
            c[t[0]] += 1
    for k, v in sorted(c.items(), key=lambda x: -x[1])[:top]:
        print(f"{v:6d} {k}")
    print("total", sum(c.values()))
    meta = s[s.index(".name:           " + m.group(1)) - 2500:s.index(".name:           " + m.group(1)) + 1500]
    for key in ("vgpr_count", "sgpr_count", "group_segment_fixed_size", "private_segment_fixed_size", "agpr_count"):
        mm = re.search(r"\." + key + r":\s+(\d+)", meta)
        if mm:
            print(key, mm.group(1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
