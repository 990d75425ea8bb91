"""Regenerate the measured tables of DESIGN.md §8 from the committed bench records:
profiles/bench_r06.jsonl (the 6 BASELINE configs, then the 20 lines of the reference integration
grid), with profiles/bench_r05.jsonl as the round-5 column. The tables sit between
<!-- BENCH_TABLE --> / <!-- INTEG_TABLE --> markers.

  python tools/design_tables.py
"""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")

CUR, PREV = "bench_r06.jsonl", "bench_r05.jsonl"
DRIVER_PREV = {"cfg2": " (driver 7718)"}


def bound_text(r):
    bm = r["bound_model"]
    sv = r.get("serial_view")
    return "%.3f of its bound (%s: %.4f ms%s); %s%.3f of dense FP4 alone" % (
        r["frac"], r["bound"], bm["bound_ms"],
        " incl. the agree's bytes" if r.get("agree_fused_in_match") else "",
        "%.3f of FP4 + keys added (`serial_view`, %.4f ms); " % (sv["frac"], sv["ms"]) if sv else "",
        r["fp4_only_view"]["frac"])


def lines(name):
    out = {}
    for ln in open(os.path.join(P, name)):
        d = json.loads(ln)
        out[d["config"]["workload"].split(":")[0]] = d
    return out


def bench_table():
    L, P0 = lines(CUR), lines(PREV)
    rows = []
    for c, label in (("cfg1", "cfg1 (8 img, 640×480, 32-bit, nxcorr 0.9)"),
                     ("cfg2", "cfg2 (33 img, 128-bit, nxcorr 0.96) — headline"),
                     ("cfg3", "cfg3 (+ min-var 2.0, subpixel 0.1)"),
                     ("cfg4", "cfg4 (40 img, 256-bit, Consistency)"),
                     ("cfg5", "cfg5 (3840×2160, 128-bit)"),
                     ("readme", "readme (3208×2200×33, min-var 2.0, subpixel 0.1)")):
        d = L[c]
        r = d["roofline"]
        h = r["hbm"]
        search = "%s %.4f ms in frame%s, %s; PMC %s%s MB (algorithmic %.1f)" % (
            "search + agree launch" if r.get("agree_fused_in_match") else "search",
            r["ms_per_launch"],
            " (search alone %.4f)" % r["search_alone_in_frame"]["ms"] if r.get("agree_fused_in_match")
            else " (%.4f back to back)" % r["search_alone_in_frame"]["back_to_back_ms"], bound_text(r),
            "search + agree, one launch: " if r.get("agree_fused_in_match") else "",
            "%.1f" % (r["traffic"] / 1e6) if r.get("traffic") else "n/a",
            r.get("algorithmic_bytes_traffic_covers", r["algorithmic_bytes"]) / 1e6)
        if c == "cfg4":
            search += "; %.3f on used bits" % r["used_bits_view"]["frac"]
        if "subpixel" in r:
            other = "subpixel %.3f ms (%.3f of spec fp32)" % (r["subpixel"]["ms"], r["subpixel"]["frac"])
        else:
            other = "transform %.4f / stack, agree %.4f" % (h["transform_ms"], h["agree_ms"])
        if c == "readme":
            other += "; one at a time %.3f ms vs ~44 ms on an RTX 4090 (README.md:90): %.1f×" % (
                d["ms_per_match_one_at_a_time"], d["vs_published"]["speedup"])
        rows.append("| %s | %.0f | %.4f | %s | %s | %.0f%s |" % (
            label, d["value"], d["ms_per_step"], search, other, P0[c]["value"], DRIVER_PREV.get(c, "")))
    head = ["| config | Mpix/s | ms/step | search stage | other stages (back to back) | round 5 Mpix/s |",
            "|---|---|---|---|---|---|"]
    return "\n".join(head + rows)


def integ_table():
    A, B = lines(CUR), lines(PREV)
    out = ["| n (bits, set) | one match at a time, ms: no subpixel / 0.25 / 0.20 / 0.15 / 0.10 | "
           "RTX 4090 ms | × | search ms in frame, frac (bound) | round 5: ×, search ms |",
           "|---|---|---|---|---|---|"]
    for n in (6, 8, 12, 16):
        names = ["integ-n%d" % n] + ["integ-n%d-s%d" % (n, s) for s in (25, 20, 15, 10)]
        d0 = A[names[0]]
        r = d0["roofline"]
        c = d0["config"]
        f = lambda m, k, fmt: fmt % A[m]["vs_published"][k]  # noqa: E731
        out.append("| %d (%d, %d) | %s | %s | %s | %.3f, %.3f (%s) | %s, %.3f |" % (
            n, c["descriptor_bits"], n * n - 2 * n + 3,
            " / ".join(f(m, "ours_ms_one_at_a_time", "%.2f") for m in names),
            " / ".join(f(m, "ms_per_match", "%.1f") for m in names),
            " / ".join(f(m, "speedup", "%.1f") for m in names),
            r["ms_per_launch"], r["frac"], r["bound"],
            " / ".join("%.1f" % B[m]["vs_published"]["speedup"] for m in names),
            B[names[0]]["roofline"]["ms_per_launch"]))
    return "\n".join(out)


def main():
    path = os.path.join(ROOT, "DESIGN.md")
    s = open(path).read()
    for tag, body in (("BENCH_TABLE", bench_table()), ("INTEG_TABLE", integ_table())):
        s, k = re.subn(r"<!-- %s -->\n.*?\n<!-- /%s -->" % (tag, tag),
                       lambda _m: "<!-- %s -->\n%s\n<!-- /%s -->" % (tag, body, tag), s, flags=re.S)
        assert k == 1, tag
    open(path, "w").write(s)
    print("DESIGN.md tables regenerated")


if __name__ == "__main__":
    main()
