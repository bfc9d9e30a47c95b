"""Map the PCs of a native crash report (glog-style '@ 0x... ' frames, the 'PC:' line and the
faulting address) to a library and offset using a /proc/self/maps dump of the same process
(bench.py RAI_DIAG_DIR).

    python tools/map_pcs.py crash.txt maps_<pid>_<tag>.txt
"""
import re
import sys


def load_maps(path):
    rows = []
    for line in open(path):
        parts = line.split()
        if len(parts) < 5:
            continue
        lo, hi = (int(x, 16) for x in parts[0].split("-"))
        off = int(parts[2], 16)
        name = parts[5] if len(parts) > 5 else "[anon]"
        rows.append((lo, hi, off, parts[1], name))
    return rows


def where(addr, rows):
    for lo, hi, off, perm, name in rows:
        if lo <= addr < hi:
            return f"{name} +0x{addr - lo + off:x} ({perm})"
    return "unmapped"


def main():
    crash, maps = sys.argv[1], sys.argv[2]
    rows = load_maps(maps)
    text = open(crash).read()
    m = re.search(r"SIGSEGV \(@(0x[0-9a-f]+)\)", text)
    if m:
        a = int(m.group(1), 16)
        print(f"fault address {m.group(1)}: {where(a, rows)}")
        near = sorted(rows, key=lambda r: min(abs(r[0] - a), abs(r[1] - a)))[:3]
        for lo, hi, off, perm, name in near:
            print(f"   nearest mapping 0x{lo:x}-0x{hi:x} {perm} {name}")
    for pc in re.findall(r"(?:PC: @|@)\s+(0x[0-9a-f]+)", text):
        print(f"{pc}: {where(int(pc, 16), rows)}")


if __name__ == "__main__":
    main()
