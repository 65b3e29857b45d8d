"""How much of the CSR encoder's per-step prep is exposed (SURVEY.md 8(d)
rows c2cli / c2low / pln): from a rocprofv3 kernel trace, the time of each
k_csr_prep (and k_encode_finalize) dispatch during which no candidate-scoring
dispatch (k_encode_prune_csr) runs on any stream, summed per grouped call
(one k_grouped_prep dispatch per call) and per coding step.

  python tools/prep_exposure.py TRACE_DIR [n_steps]

Prints one line per kernel family and a JSON summary on the last line."""
import csv
import glob
import json
import sys


def load(d):
    ev = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ev.sort()
    return ev


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def uncovered(s, e, cover):
    """Length of [s, e) not inside the (sorted, disjoint) cover intervals."""
    left = e - s
    for a, b in cover:
        if b <= s:
            continue
        if a >= e:
            break
        left -= min(b, e) - max(a, s)
    return left


def main():
    d = sys.argv[1]
    n_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    ev = load(d)
    calls = sum(1 for _, _, n in ev if "k_grouped_prep" in n) or 1
    scoring = union([(s, e) for s, e, n in ev if "k_encode_prune_csr" in n])
    out = {"calls": calls, "n_steps": n_steps}
    for fam in ("k_csr_prep", "k_encode_finalize", "k_encode_prune_csr"):
        iv = [(s, e) for s, e, n in ev if fam in n]
        if not iv:
            continue
        tot = sum(e - s for s, e in iv)
        if fam == "k_encode_prune_csr":
            exp = 0
        else:
            exp = sum(uncovered(s, e, scoring) for s, e in iv)
        out[fam] = {"dispatches": len(iv), "us_per_call": tot / calls / 1e3,
                    "exposed_us_per_call": exp / calls / 1e3,
                    "exposed_us_per_step": exp / calls / n_steps / 1e3}
        print(f"{fam:20s} {len(iv):6d} dispatches, {tot / calls / 1e3:9.1f} us per call, "
              f"exposed (no scoring dispatch running) {exp / calls / 1e3:8.1f} us per call = "
              f"{exp / calls / n_steps / 1e3:6.2f} us per step")
    # the calls' device span: first to last dispatch of each call
    starts = [s for s, _, n in ev if "k_grouped_prep" in n]
    spans, busy = [], []
    for i, s0 in enumerate(starts):
        s1 = starts[i + 1] if i + 1 < len(starts) else max(e for _, e, _ in ev) + 1
        sel = [(s, e) for s, e, n in ev if s0 <= s < s1]
        spans.append(max(e for _, e in sel) - s0)
        busy.append(sum(b - a for a, b in union(sel)))
    out["call_span_us"] = sum(spans) / len(spans) / 1e3
    out["call_busy_us"] = sum(busy) / len(busy) / 1e3
    if "k_csr_prep" in out:
        out["prep_exposed_frac_of_span"] = out["k_csr_prep"]["exposed_us_per_call"] / \
            out["call_span_us"]
    print(f"call device span {out['call_span_us']:.1f} us, busy {out['call_busy_us']:.1f} us")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
