"""Summarise a tools/profile_round.sh run into small committed files under profiles/.

One env step is several launches (staged: k_soccer_rows, k_pgs_groups twice — main and global-B
launch —, k_soccer_finish, k_soccer_fixup; monolithic: k_soccer<.., 0>): the step's kernel time
is the sum of their rocprof averages times their calls per step, and its HBM traffic the same
sum over their per-dispatch counter means. HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB, collected in separate passes; on gfx950 FETCH_SIZE counts half the bytes of a wide
coalesced read, so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (raw values kept too).
"""
import csv
import glob
import json
import os
import shutil
import sys

STEP_KERNELS = ["k_soccer_rows", "k_pgs_groups", "k_soccer_bank_finish", "k_soccer_finish", "k_soccer_fixup", "k_soccer_settle",
                "k_rk_rows", "k_rk_finish", "k_rk_settle", "k_pk_rows", "k_pk_bank_finish", "k_pk_finish", "k_pk_settle",
                "k_soccer<float, 0>",
                "k_soccer<double, 0>", "k_bipedal<float, 0, true>", "k_bipedal<float, 0, false>",
                "k_parkour<float, 0>", "k_parkour<float, 0, true>", "k_parkour<float, 0, false>",
                "k_martial<float, 0, true>", "k_martial<float, 0, false>",
                "k_assembly<double, 0, true>", "k_assembly<double, 0, false>",
                "k_parkour<double, 0, true>", "k_parkour<double, 0, false>", "k_martial<double, 0, true>",
                "k_martial<double, 0, false>", "k_dancing<double, 0, true>", "k_dancing<double, 0, false>",
                "k_construction<double, 0>", "k_construction<double, 0, true>", "k_construction<double, 0, false>"]


def step_kernel(name):
    for k in STEP_KERNELS:
        if k in name:
            return k
    return None


def find(d, pat):
    g = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return g[0] if g else None


def counter_means(d, counter):
    """mean counter value per dispatch, per step kernel"""
    f = find(d, "*counter_collection.csv")
    if not f:
        return {}
    per = {}
    for r in csv.DictReader(open(f)):
        k = step_kernel(r.get("Kernel_Name", ""))
        if not k or r.get("Counter_Name") != counter:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per.setdefault(k, {})
        per[k][key] = per[k].get(key, 0.0) + float(r["Counter_Value"])
    # the settle kernel's reset() dispatch (outside the timed steps) moves the whole batch's
    # settle traffic: its per-step value is the median dispatch
    return {k: (sorted(v.values())[len(v) // 2] if "settle" in k else sum(v.values()) / len(v))
            for k, v in per.items() if v}


def main(out, tag):
    summ = os.path.join(out, "summary")
    os.makedirs(summ, exist_ok=True)
    stats = find(os.path.join(out, "trace"), "*kernel_stats.csv")
    res = {"tag": tag, "kernels": {}}
    if stats:
        shutil.copy(stats, os.path.join(summ, f"{tag}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats)):
            k = step_kernel(r["Name"])
            if k:
                calls, tot, mx = int(r["Calls"]), float(r["TotalDurationNs"]), float(r["MaxNs"])
                avg = tot / calls
                if "settle" in k and calls > 1:
                    # the settle kernel's longest call is reset() (every env settled, banks
                    # prefilled), outside the timed steps; the per-step calls are the fallback
                    avg = (tot - mx) / (calls - 1)
                    calls -= 1
                res["kernels"][k] = {"avg_ms": avg / 1e6, "calls": calls, "pct": float(r["Percentage"])}
        # a kernel may run more than once per step (the staged solver: main launch + global-B
        # launch; the RK4 pipeline: four of each stage kernel); the step count is the fewest calls
        # of any step kernel
        nstep = min(v["calls"] for v in res["kernels"].values()) if res["kernels"] else 1
        for v in res["kernels"].values():
            v["per_step"] = v["calls"] / nstep
        res["rocprof_step_ms"] = sum(v["avg_ms"] * v["per_step"] for v in res["kernels"].values())
    bj = os.path.join(out, "bench_under_rocprof.json")
    if os.path.exists(bj):
        line = [x for x in open(bj).read().splitlines() if x.startswith("{")]
        if line:
            b = json.loads(line[-1])
            shutil.copy(bj, os.path.join(summ, f"{tag}_bench_under_rocprof.json"))
            res["bench_step_ms_same_run"] = b["roofline"]["launch_ms"]
            res["envs"] = b["config"].get("envs_per_gpu", b["config"].get("envs_per_task"))
            res["precision"] = b["dtype"]
            # the mixed run (every task's step kernels on four streams): mode "mixed"
            res["mode"] = "mixed" if "envs_per_task" in b["config"] else b["config"].get("step_kernels", "staged")
            res["task"] = b["config"]["workload"].split("_env")[0]
    fetch = counter_means(os.path.join(out, "pmc_fetch"), "FETCH_SIZE")
    write = counter_means(os.path.join(out, "pmc_write"), "WRITE_SIZE")
    if fetch and write:
        for k in set(fetch) | set(write):
            kk = res["kernels"].setdefault(k, {})
            kk["fetch_kib_raw"] = fetch.get(k, 0.0)
            kk["write_kib_raw"] = write.get(k, 0.0)
            kk["hbm_bytes"] = (2 * fetch.get(k, 0.0) + write.get(k, 0.0)) * 1024
        res["hbm_bytes_per_step"] = sum(v.get("hbm_bytes", 0.0) * v.get("per_step", 1.0) for v in res["kernels"].values())
        res["correction"] = "(2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md §HBM"
    with open(os.path.join(summ, f"{tag}_pmc.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
