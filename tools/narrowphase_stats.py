"""How often each narrowphase branch fires at bench conditions (CPU oracle; test infrastructure).

Runs the soccer CPU baseline of bench.py (oracle/mjref.c physics + oracle/soccer_logic.py, U(-150,
150) actions, same-step autoreset) and prints the oracle's branch counters: capsule-box pairs with
one / two contacts, capsule-capsule general / parallel branch, box-box pairs by contact count.

usage: python tools/narrowphase_stats.py [envs] [steps]  ->  JSON on stdout
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(envs: int = 16, steps: int = 500) -> dict:
    import bench
    from oracle.mjref import narrowphase_stats
    narrowphase_stats(reset=True)
    base = bench.cpu_baseline(envs, steps, seed=0)
    st = narrowphase_stats()
    cb = st["capsule_box_1"] + st["capsule_box_2"]
    out = {"task": "humanoid_soccer", "envs": envs, "steps_per_env": steps, "env_steps": envs * steps,
           "actions": "U(-150, 150), same-step autoreset (bench.py cpu_baseline)", "counters": st,
           "capsule_box_pairs_in_contact": cb,
           "capsule_box_two_contact_share": st["capsule_box_2"] / cb if cb else None,
           "capsule_capsule_parallel_share": st["capsule_capsule_parallel"] / max(1, st["capsule_capsule"] +
                                                                                st["capsule_capsule_parallel"]),
           "oracle_env_steps_per_s": round(base["value"], 1)}
    return out


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:3]]
    print(json.dumps(main(*a)))
