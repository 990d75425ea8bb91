"""Append the last JSON line of stdin, tagged, to a JSON-lines file (GPU session helper).

  python bench.py ... | python tools/jl.py OUT.jsonl key=value [key=value ...]
Keeps bench lines' headline fields (value, ms_per_step, one-at-a-time latency, the roofline's
launch time / frac / bound, the host path) so A/B records stay small."""
import json
import sys

KEEP = ("config", "value", "ms_per_step", "ms_per_match_one_at_a_time", "frames_in_flight", "steps")


def main():
    out, tags = sys.argv[1], dict(a.split("=", 1) for a in sys.argv[2:])
    lines = [l for l in sys.stdin.read().splitlines() if l.startswith("{")]
    if not lines:
        raise SystemExit("no JSON line on stdin")
    d = json.loads(lines[-1])
    rec = dict(tags)
    if "metric" in d:  # a bench.py line
        rec.update({k: d[k] for k in KEEP if k in d})
        rec["config"] = d["config"]["workload"].split(":")[0]
        r = d.get("roofline") or {}
        rec.update({"roof_ms": r.get("ms_per_launch"), "roof_frac": r.get("frac"),
                    "roof_bound": r.get("bound")})
        if d.get("host_path"):
            rec["host_ms"] = d["host_path"]["ms_per_match"]
        if d.get("root_load"):
            rec["ingress"] = d["root_load"]
        rec["rows"] = d["config"].get("rows_per_rank")
    else:
        rec.update(d)
    with open(out, "a") as f:
        f.write(json.dumps(rec) + "\n")
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
