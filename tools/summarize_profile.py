#!/usr/bin/env python3
"""Turn a gpurun_out/prof directory (tools/profile.sh) into committed
profiles/: the rocprofv3 kernel stats, per-kernel PMC byte counts and the
calibrated per-launch HBM traffic of the SpMV (profiles/spmv_traffic.json,
read by bench.py for roofline.traffic).

    python tools/summarize_profile.py gpurun_out/prof r01 [grid] [n_gpus]
"""
import csv
import json
import os
import re
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    """'void mx::spmv_sell_kernel<3, true, 7, false>(long, ...)' -> 'spmv_sell_kernel<3,true,7,false>'."""
    n = re.sub(r"^void\s+", "", name).replace("(anonymous namespace)::", "")
    n = n.split("(")[0].replace("mx::", "").replace(" ", "")
    return n


def pmc(path):
    per = {}
    for r in csv.DictReader(open(path)):
        per.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return per


def main():
    src, tag = sys.argv[1], sys.argv[2]
    grid = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    ngpu = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    # per-launch durations from the trace.  Launches shorter than NOOP_US are
    # dropped: a launch enqueued after the solve has stopped exits on the done
    # flag in a few us (the library now launches only the max_it remainder,
    # but a solve that converges inside a batch still has some), and would
    # drag the mean and median of the working launches down
    NOOP_US = 10.0
    alld, durs, dropped = {}, {}, {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
        alld.setdefault(short(r["Kernel_Name"]), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, ts in alld.items():
        work = len(ts) >= 10 and statistics.median(ts) >= 2 * NOOP_US   # an iteration kernel with some no-op launches
        keep = [t for t in ts if not (work and t < NOOP_US)]
        if len(keep) < len(ts):
            dropped[k] = len(ts) - len(keep)
        durs[k] = keep
    fetch = pmc(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write = pmc(os.path.join(src, "write", "run_counter_collection.csv"))
    calib = pmc(os.path.join(src, "calib", "run_counter_collection.csv"))
    known = (1 << 27) * 8
    # the calibration runs 3 launches at 8 B/lane then 3 at 16 B/lane
    c8 = next((v for k, v in calib.items() if k.startswith("stream_read_kernel<8")), [])
    c16 = next((v for k, v in calib.items() if k.startswith("stream_read_kernel<16")), [])
    f8 = known / (statistics.median(c8) * 1024) if c8 else None
    f16 = known / (statistics.median(c16) * 1024) if c16 else None
    m = grid ** 3 // ngpu
    nnz = 7 * grid ** 3 - 6 * grid ** 2
    ghosts = 0 if ngpu == 1 else (grid * grid * (1 if ngpu == 2 else 2))
    # the streamed layout's bytes (bench.py spmv_format_bytes): value codes at one
    # byte per slot (7 offsets -> 8 B/row), x once, y once, slice metadata, A_o;
    # SURVEY.md §8d's CSR figure in csr_bytes
    csr_bytes = 12 * nnz // ngpu + 4 * (m + 1) + 8 * (m + ghosts) + 8 * m
    spmv_alg = 8 * m + 8 * (m + ghosts) + 8 * m + 16 * ((m + 63) // 64) + (12 * ghosts + 4 * (m + 1) if ghosts else 0)
    alg = spmv_alg + 32 * m          # SPMV_CG: + r read, x read/write, p_i write
    out = {}
    lines = [f"# {tag}: rocprofv3 summary (3D 7-pt Poisson {grid}^3, N={ngpu}, bench.py --steps 50)", "",
             "| kernel | calls | working launches | mean us (working) | median us (working) | % time | FETCH_SIZE KB (raw, median) | WRITE_SIZE KB (median) |",
             "|---|---|---|---|---|---|---|---|"]
    for r in stats[:14]:
        k = short(r["Name"])
        fk = statistics.median(fetch[k]) if k in fetch else None
        wk = statistics.median(write[k]) if k in write else None
        w = durs.get(k, [])
        med = statistics.median(w) if w else float("nan")
        mean = statistics.mean(w) if w else float("nan")
        lines.append(f"| {k} | {r['Calls']} | {len(w)} | {mean:.1f} | {med:.1f} | {float(r['Percentage']):.1f} | "
                     f"{'' if fk is None else f'{fk:.0f}'} | {'' if wk is None else f'{wk:.0f}'} |")
    if dropped:
        lines += ["", "No-op launches (< 10 us, after a stop) dropped from mean/median: " +
                  ", ".join(f"{k} {n}" for k, n in sorted(dropped.items()))]
    # the solve's MatMult: the SpMV kernel with the most device time (the
    # CG-fused SPMV_CG <3,...> at <= 3M rows/rank, SPMV_DOT <2,...> above:
    # the general kernel or the lean row-pair / z-march kernels)
    # (CG mode 5: the residual update spmv_pair_zm_kernel<7,...> -- SPMV_RUPD --
    # is the roofline kernel, keyed "/mode5")
    # (from 2^23 rows: its two-lines-per-wave form spmv_pair_zm2l_kernel)
    cands = [k for k in fetch if k.startswith(("spmv_sell_kernel<3,", "spmv_sell_kernel<2,", "spmv_pair_zm_kernel<7,",
                                               "spmv_pair_zm2l_kernel<", "spmv_pair_zm_kernel<2,",
                                               "spmv_pair_lean_kernel<2,"))]
    sp = max(cands, key=lambda k: sum(durs.get(k, [0.0]))) if cands else None
    if sp and not sp.startswith("spmv_sell_kernel<3,"):
        alg = spmv_alg
    # the profiled bench's own figure (bench.py spmv_format_bytes: code-block
    # dictionary, value codes) when its JSON line is in the trace log
    js = []
    try:
        with open(os.path.join(src, "trace.log")) as f:
            js = [json.loads(ln) for ln in f if ln.startswith("{")]
        if js and js[-1].get("roofline", {}).get("bytes_per_launch"):
            alg = js[-1]["roofline"]["bytes_per_launch"]
    except (OSError, ValueError):
        pass
    if sp in fetch and sp in write:
        fr = statistics.median(fetch[sp]) * 1024
        wr = statistics.median(write[sp]) * 1024
        corr = f16 if f16 else 2.0
        traffic = fr * corr + wr
        out[f"{grid}^3/N{ngpu}" + ("/mode5" if sp.startswith(("spmv_pair_zm_kernel<7,", "spmv_pair_zm2l_kernel<"))
                                   else "")] = {
            "bytes_per_launch": round(traffic), "fetch_bytes_raw": round(fr), "write_bytes": round(wr),
            "fetch_correction": round(corr, 4), "calib_8B_per_lane": f8 and round(f8, 4),
            "calib_16B_per_lane": f16 and round(f16, 4), "algorithmic_bytes": alg,
            "traffic_over_algorithmic": round(traffic / alg, 4), "kernel": sp, "csr_bytes": csr_bytes,
            "median_launch_us": round(statistics.median(durs[sp]), 1) if sp in durs else None,
            "source": f"profiles/{tag}_summary.md"}
        lines += ["", f"{sp} per launch: FETCH_SIZE {fr/1e6:.1f} MB raw x {corr:.3f} (calibrated, 16 B/lane NT stream; "
                  f"8 B/lane factor {f8 and round(f8, 3)}) + WRITE_SIZE {wr/1e6:.1f} MB = {traffic/1e6:.1f} MB "
                  f"vs {alg/1e6:.1f} MB algorithmic ({traffic/alg:.3f}x)."]
    # beside the roofline kernel: the direction update (mode 5's longest
    # kernel, cg_pb_kernel<JM, 4>) and the streamed-values MatMult of bench.py's
    # spmv_general leg (spmv_pair_zmf64_kernel), each against the bench line's
    # own algorithmic bytes
    js_last = js[-1] if js else {}
    corr = f16 if f16 else 2.0
    extra = []
    dom = (js_last.get("roofline") or {}).get("dominant_kernel") or {}
    gen = js_last.get("spmv_general") or {}
    xb = js_last.get("cg_xbatch") or 4
    pbk = [k for k in fetch if k.startswith("cg_pb_kernel<") and k.endswith(f",{xb}>")]
    if pbk and dom.get("bytes_per_launch"):
        extra.append((f"{grid}^3/N{ngpu}/pb", max(pbk, key=lambda k: sum(durs.get(k, [0.0]))), dom["bytes_per_launch"]))
    gk = [k for k in fetch if k.startswith("spmv_pair_zmf64_kernel<2,")]
    if gk and gen.get("streamed_bytes"):
        extra.append((f"varcoef{grid}^3/N{ngpu}", gk[0], gen["streamed_bytes"]))
    for key, k, a in extra:
        if k in fetch and k in write:
            # the direction update's launches differ (every xb-th one carries the
            # x batch): its algorithmic bytes are a per-launch mean, so is its traffic
            agg = statistics.mean if key.endswith("/pb") else statistics.median
            fr, wr = agg(fetch[k]) * 1024, agg(write[k]) * 1024
            t = fr * corr + wr
            out[key] = {"bytes_per_launch": round(t), "fetch_bytes_raw": round(fr), "write_bytes": round(wr),
                        "fetch_correction": round(corr, 4), "algorithmic_bytes": a,
                        "traffic_over_algorithmic": round(t / a, 4), "kernel": k,
                        "median_launch_us": round(statistics.median(durs[k]), 1) if k in durs else None,
                        "source": f"profiles/{tag}_summary.md"}
            lines += [f"{k} per launch ({key}): FETCH_SIZE {fr/1e6:.1f} MB raw x {corr:.3f} + WRITE_SIZE "
                      f"{wr/1e6:.1f} MB = {t/1e6:.1f} MB vs {a/1e6:.1f} MB algorithmic ({t/a:.3f}x)."]
    lines += ["", "Produced by: `bash tools/gpu_run.sh <tag> prof` (tools/profile.sh: rocprofv3 --kernel-trace --stats, "
              "then --pmc FETCH_SIZE and --pmc WRITE_SIZE passes of `bench.py --steps 50 --warmup 5 --no-cpu "
              "--no-solve --no-asm`, and the tools/calib_stream.py calibration pass), then "
              f"`python tools/summarize_profile.py {src} {tag} {grid} {ngpu}`."]
    with open(os.path.join(dst, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    tj = os.path.join(dst, "spmv_traffic.json")
    cur = json.load(open(tj)) if os.path.exists(tj) else {}
    cur.update(out)
    json.dump(cur, open(tj, "w"), indent=1, sort_keys=True)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
