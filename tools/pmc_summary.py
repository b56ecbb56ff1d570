"""Summarise a round's PMC passes (tools/gpu_pmc_rNN.sh -> gpurun_out/pmcN) into
profiles/<tag>_pmc_traffic.json (bench.py reads `traffic_bytes` from the newest one) and
profiles/<tag>_pmc_sq.json.  Usage: pmc_summary.py SRC_DIR TAG (default gpurun_out/pmc2 r02).
FETCH_SIZE / WRITE_SIZE are in KB; FETCH_SIZE is doubled (MI355X_MICROARCH.md: on gfx950 it
reports half of a wide streaming read)."""
import collections
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
SRC = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "pmc2")
TAG = sys.argv[2] if len(sys.argv) > 2 else "r02"


# pass directories: round 2 numbered them, later rounds name them <mode>_<group>
_R02 = {("wino_one", "sq1"): "p1_wino_one", ("wino_one", "sq2"): "p2_wino_one",
        ("mix", "fetch"): "p3_mix", ("mix", "write"): "p4_mix", ("ns", "fetch"): "p5_ns",
        ("ns", "write"): "p6_ns", ("ns", "sq"): "p7_ns", ("upfirdn", "fetch"): "p8_upfirdn",
        ("upfirdn", "write"): "p9_upfirdn"}


def pdir(mode, grp):
    return _R02[(mode, grp)] if TAG == "r02" else f"{mode}_{grp}"


def rows(pattern):
    """all counter rows of a pass, in dispatch order"""
    f = glob.glob(os.path.join(SRC, pattern, "pmc_counter_collection.csv"))[0]
    return sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))


def step_bytes(mode, counter):
    """KB of `counter` summed over the dispatches between the last two marker dispatches
    (fused_bias_act_kernel, tools/prof_steps.py), and the number of dispatches; read from the
    pass's reduced JSON when the GPU run already reduced (and dropped) the per-dispatch CSV"""
    red = os.path.join(SRC, pdir(mode, counter.split("_")[0].lower()) + ".json")
    if os.path.exists(red):
        d = json.load(open(red))
        # a pass reduced on the box records the kernel sources it ran; one from another tree
        # (a pass that crashed this time leaves the previous run's file) is not this tree's
        want = provenance("step")["src_sha1"]
        assert d.get("src_sha1") == want, (mode, counter, "stale pass", d.get("src_sha1"), want)
        return d["sum_kb"], d["dispatches"]
    per = collections.OrderedDict()
    for r in rows(pdir(mode, counter.split("_")[0].lower())):
        d = per.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "v": 0.0})
        if r["Counter_Name"] == counter:
            d["v"] += float(r["Counter_Value"])
    ids = list(per)
    marks = [i for i, d in enumerate(per.values()) if "fused_bias_act_kernel<double>" in d["name"]]
    assert len(marks) >= 2, (mode, counter, len(marks))
    a, b = marks[-2], marks[-1]
    inside = [per[ids[i]]["v"] for i in range(a + 1, b)]
    return sum(inside), len(inside)


def load(pattern, keep):
    f = glob.glob(os.path.join(SRC, pattern, "pmc_counter_collection.csv"))[0]
    agg = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if keep(r["Kernel_Name"]):
            agg[int(r["Dispatch_Id"])][r["Counter_Name"]] = \
                agg[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            agg[int(r["Dispatch_Id"])]["_grid"] = int(r["Grid_Size"])
            agg[int(r["Dispatch_Id"])]["_kernel"] = r["Kernel_Name"].split("(")[0]
    return [agg[d] for d in sorted(agg)]


def provenance(key, recs=()):
    """What bench.py checks before it attaches an entry to a live measurement: the sha1 of
    the kernel sources the counted dispatches were built from (this tree = the tree the GPU
    pass ran) and the kernel symbols counted."""
    import bench
    src = next(v for k, v in bench.PMC_SOURCES.items() if key.startswith(k))
    out = {"src_sha1": bench.src_sha1(src)}
    names = sorted({r["_kernel"] for r in recs if "_kernel" in r})
    if names:
        out["kernels"] = names
    return out


def main():
    import bench
    wino = lambda k: "wino_f23" in k
    mix_f = [d["FETCH_SIZE"] for d in load(pdir("mix", "fetch"), wino)]
    mix_w = [d["WRITE_SIZE"] for d in load(pdir("mix", "write"), wino)]
    n = sum(r[3] + r[4] for r in bench.WINO_MIX)
    assert len(mix_f) == len(mix_w) == n, (len(mix_f), len(mix_w), n)
    out = {"wino_pre_mix": {
        "traffic_bytes": 1024.0 * (2 * sum(mix_f) + sum(mix_w)),
        "fetch_bytes_x2": 2048.0 * sum(mix_f), "write_bytes": 1024.0 * sum(mix_w),
        "launches": n, "note": "one NCSN++ 128^2 forward's PRE-conv mix at B=64 (bench.WINO_MIX)",
        **provenance("wino_pre_mix", load(pdir("mix", "fetch"), wino))}}
    up = lambda k: "upfirdn" in k
    uf = load(pdir("upfirdn", "fetch"), up)
    uw = load(pdir("upfirdn", "write"), up)
    for i, (name, *_rest) in enumerate(bench.UPFIRDN_SHAPES):
        f = sum(d["FETCH_SIZE"] for d in uf[3 * i:3 * i + 3]) / 3
        w = sum(d["WRITE_SIZE"] for d in uw[3 * i:3 * i + 3]) / 3
        out["upfirdn2d " + name] = {"traffic_bytes": 1024.0 * (2 * f + w),
                                    "fetch_bytes_x2": 2048.0 * f, "write_bytes": 1024.0 * w,
                                    **provenance("upfirdn2d", uf[3 * i:3 * i + 3])}
    ns = lambda k: "k_fused" in k
    nf = load(pdir("ns", "fetch"), ns)
    nw = load(pdir("ns", "write"), ns)
    f = sum(d["FETCH_SIZE"] for d in nf) / 3
    w = sum(d["WRITE_SIZE"] for d in nw) / 3
    out["ns_step full step B256 192^2"] = {"traffic_bytes": 1024.0 * (2 * f + w),
                                            "fetch_bytes_x2": 2048.0 * f, "write_bytes": 1024.0 * w,
                                            "note": "both fused launches of one full step",
                                            **provenance("ns_step", nf)}
    if TAG != "r02":
        units = {"train": "step", "cifar": "step", "pinn": "step", "dps": "nfe"}
        for mode, unit in units.items():
            try:
                f, nf = step_bytes(mode, "FETCH_SIZE")
                w, nw = step_bytes(mode, "WRITE_SIZE")
            except (IndexError, AssertionError) as e:
                print("no step passes for", mode, e)
                continue
            out["step " + mode] = {"traffic_bytes": 1024.0 * (2 * f + w),
                                   "fetch_bytes_x2": 2048.0 * f, "write_bytes": 1024.0 * w,
                                   "dispatches": [nf, nw],
                                   "note": f"all kernels of one bench {mode} {unit} "
                                           "(tools/prof_steps.py markers)",
                                   **provenance("step")}
    out["_note"] = (f"rocprofv3 --pmc passes (tools/gpu_pmc_{TAG}.sh over tools/prof_r02.py); "
                    "FETCH_SIZE x2 (gfx950) + WRITE_SIZE, KB -> bytes")
    json.dump(out, open(os.path.join(REPO, "profiles", f"{TAG}_pmc_traffic.json"), "w"), indent=1)
    sq = {}
    one = [d for d in load(pdir("wino_one", "sq1"), wino)]
    one2 = [d for d in load(pdir("wino_one", "sq2"), wino)]
    last = dict(one[-1]); last.update(one2[-1])
    waves = last["_grid"] / 64
    last["derived"] = {
        "mfma_busy_frac_of_simd_cycles": last["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * last["GRBM_GUI_ACTIVE"] / 8),
        "lds_bank_conflict_frac": last["SQ_LDS_BANK_CONFLICT"] / max(1.0, last["SQ_LDS_IDX_ACTIVE"]),
        "wait_inst_any_frac": last["SQ_WAIT_INST_ANY"] / last["SQ_WAVE_CYCLES"],
        "wait_any_frac": last["SQ_WAIT_ANY"] / last["SQ_WAVE_CYCLES"],
        "valu_per_mfma": last["SQ_INSTS_VALU"] / last["SQ_INSTS_MFMA"],
        "waves": waves}
    sq["wino_pre_stats 128->128@128 B=16 (one dispatch)"] = last
    nsq = load(pdir("ns", "sq"), ns)
    sq["ns_step launches (3 full steps)"] = {"runs": nsq, **provenance("ns_step", nsq)}
    sq["_note"] = ("SQ_* wave counters in quad-cycles except SQ_VALU_MFMA_BUSY_CYCLES (cycles, = 32 per "
                   "v_mfma_f32_16x16x4_f32); GRBM_GUI_ACTIVE summed over the 8 XCDs; MFMA busy "
                   "fraction = MFMA busy cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)")
    json.dump(sq, open(os.path.join(REPO, "profiles", f"{TAG}_pmc_sq.json"), "w"), indent=1)
    print(json.dumps({k: v.get("traffic_bytes") for k, v in out.items() if isinstance(v, dict)}, indent=1))
    print(json.dumps(last["derived"], indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[3] == "reduce-step":
        # on the GPU box: reduce one step pass (argv[4] = mode, argv[5] = counter) to JSON
        kb, n = step_bytes(sys.argv[4], sys.argv[5])
        json.dump({"sum_kb": kb, "dispatches": n, "src_sha1": provenance("step")["src_sha1"]},
                  open(os.path.join(SRC, pdir(sys.argv[4], sys.argv[5].split("_")[0].lower())
                                    + ".json"), "w"))
        print("reduced", sys.argv[4], sys.argv[5], kb, n)
    else:
        main()
