"""Per-kernel register / occupancy / LDS summary of a hipcc `-S` device assembly file.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S engine.hip -o e.s
    python scripts/isa_stats.py e.s [substring-filter]
"""
import re
import subprocess
import sys


def demangle(names):
    try:
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt"], input="\n".join(names),
                             capture_output=True, text=True, check=True).stdout.splitlines()
        return out if len(out) == len(names) else names
    except Exception:
        return names


def parse(path):
    rows, cur = [], None
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr", r"; NumVgprs: (\d+)"), ("total", r"; TotalNumVgprs: (\d+)"),
                         ("occ", r"; Occupancy: (\d+)"), ("lds", r"; LDSByteSize: (\d+)"),
                         ("scratch", r"; ScratchSize: (\d+)")):
            mm = re.search(pat, line)
            if mm and key not in cur:
                cur[key] = int(mm.group(1))
    return rows


def main():
    rows = parse(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    names = demangle([r["name"] for r in rows])
    for r, n in zip(rows, names):
        n = n.replace("void ddl::", "").replace("ddl::", "")
        n = re.sub(r"\(.*\)$", "", n)
        if filt and filt not in n:
            continue
        print(f"{r.get('vgpr', '?'):>4} {r.get('total', '?'):>4} occ={r.get('occ', '?')} "
              f"lds={r.get('lds', '?'):>6} scr={r.get('scratch', 0)}  {n}")


if __name__ == "__main__":
    main()
