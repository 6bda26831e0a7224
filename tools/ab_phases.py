"""Summarise an alternated phase-timing A/B log (lines 'round R lib L n N' each followed by
tools/phase_timing.py's JSON line): per (lib, n), each phase's runs and the total."""
import collections
import json
import re
import sys

res = collections.defaultdict(list)
cur = None
for line in open(sys.argv[1]):
    m = re.match(r"round (\d+) lib (\S+) n (\d+)", line)
    if m:
        cur = (m.group(2), int(m.group(3)))
    elif line.startswith("{") and cur:
        res[cur].append(json.loads(line)["phases"])
phases = sys.argv[2].split(",") if len(sys.argv) > 2 else ["reduce", "combine", "pairing"]
for k, v in sorted(res.items()):
    print(k, " ".join("%s=%s" % (ph, "/".join("%.3f" % x[ph] for x in v)) for ph in phases),
          "total", "/".join("%.3f" % sum(x.values()) for x in v))
