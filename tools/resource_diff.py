"""Compare the per-kernel resource usage of two hipcc -Rpass-analysis=kernel-resource-usage
logs (VGPRs, AGPRs, SGPRs, scratch, occupancy), e.g. before / after a source change:

    hipcc ... -c search_mx.hip -Rpass-analysis=kernel-resource-usage 2> new.txt
    python tools/resource_diff.py old.txt new.txt [--drop-last-bool]

--drop-last-bool maps a new kernel whose template list gained a trailing bool parameter
onto the old name (only the `false` instantiations are compared)."""
import re
import subprocess
import sys

KEYS = ("VGPRs", "AGPRs", "TotalSGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]")


def parse(path):
    out, cur = {}, None
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+([^:]+): (\d+)", line)
        if m and cur:
            out[cur][m.group(1).strip()] = int(m.group(2))
    return out


def main():
    old, new = parse(sys.argv[1]), parse(sys.argv[2])
    drop = "--drop-last-bool" in sys.argv
    changed = 0
    for name, v in sorted(new.items()):
        key = name
        if drop:
            if not re.search(r", false>\(", name):
                continue
            key = re.sub(r", false>\(", ">(", name)
        o = old.get(key)
        if o is None:
            print("new only:", name[:120])
            continue
        d = {k: (o.get(k), v.get(k)) for k in KEYS if o.get(k) != v.get(k)}
        if d:
            changed += 1
            print(name[:120], d)
    print("%d kernels compared, %d changed" % (len(new), changed))


if __name__ == "__main__":
    main()
