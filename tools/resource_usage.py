"""Tabulate hipcc -Rpass-analysis=kernel-resource-usage output (build/resource_usage.txt)."""
import re, subprocess, sys
path = sys.argv[1] if len(sys.argv) > 1 else "build/resource_usage.txt"
rows, cur = [], None
for line in open(path):
    m = re.search(r"(?:remark: )?\S+:\d+:\d+: (?:remark: )?(.*?) \[-Rpass", line)
    if not m:
        continue
    txt = m.group(1).strip()
    if txt.startswith("Function Name:"):
        name = txt.split(":", 1)[1].strip()
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except Exception:
            pass
        cur = {"name": name}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
keys = ["VGPRs", "AGPRs", "TotalSGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill", "VGPRs Spill", "LDS Size [bytes/block]"]
print("%-70s %s" % ("kernel", " ".join(k.split()[0][:8].rjust(8) for k in keys)))
for r in rows:
    n = re.sub(r"\(anonymous namespace\)::", "", r["name"])
    print("%-70s %s" % (n[:70], " ".join(str(r.get(k, "-")).rjust(8) for k in keys)))
