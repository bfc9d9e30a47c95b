"""C3 HBM traffic from the two per-kernel PMC passes of tools/c3_pmc.sh (one eager C3 update,
1024 envs x 128 steps, B = 256, 4 epochs = 2,048 optimizer steps).

    python tools/c3_traffic.py <FETCH_SIZE.json> <WRITE_SIZE.json> <out.json> [--lib <librai_amd.so>]

Bytes per kernel = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; the x2 is MI355X_MICROARCH.md's gfx950
correction for wide streaming reads, exact for 16-B-per-lane loads and uncalibrated for narrower
ones; Infinity-Cache hits count as fetches).  Kernels dispatched at least once per optimizer step
(>= 2,048 dispatches) form the minibatch step; the rest of the update's kernels (rollout forward,
GAE, per-epoch gathers) are added once.  The bench's own extra measurements in the same process (the
bandwidth-regime GAE, gae_stream_kernel), MIOpen find-mode trial kernels (present in the FETCH
pass only: the WRITE pass reuses the find database) and TunableOp's GEMM tuning trials (hipBLASLt kernels
dispatched fewer times than there are optimizer steps) are excluded.
"""
import hashlib
import json
import os
import sys

STEPS = int(os.environ.get("TRAFFIC_STEPS", "2048"))  # minibatch steps per update (C3 2,048; C5 86)


def main():
    f = json.load(open(sys.argv[1]))["kernels"]
    w = json.load(open(sys.argv[2]))["kernels"]
    kernels, step_b, upd_b = {}, 0.0, 0.0
    dropped = 0.0
    for k, we in w.items():
        if "gae_stream_kernel" in k:
            continue
        if k.startswith("Cijk") and we["dispatches"] < STEPS:
            # hipBLASLt solutions TunableOp times while tuning, inside the profiled (first) update: 1,200+
            # GEMM kernels, ~2.6 TB.  The rollout's fc-forward GEMMs (129 per update) go with them.
            dropped += 2.0 * f.get(k, {}).get("FETCH_SIZE", 0.0) * 1024 + we.get("WRITE_SIZE", 0.0) * 1024
            continue
        fe = f.get(k, {})
        n = we["dispatches"]
        fetch = 2.0 * fe.get("FETCH_SIZE", 0.0) * 1024 * (n / max(fe.get("dispatches", n), 1))
        write = we.get("WRITE_SIZE", 0.0) * 1024
        tot = fetch + write
        per_step = n >= STEPS
        kernels[k] = {"dispatches": n, "bytes_per_launch": round(tot / n), "fetch_x2_per_launch": round(fetch / n),
                      "write_per_launch": round(write / n), "per_optimizer_step": per_step}
        if per_step:
            step_b += tot / STEPS
        else:
            upd_b += tot
    top = sorted(kernels.items(), key=lambda kv: -kv[1]["bytes_per_launch"] * kv[1]["dispatches"])
    libp = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "..", "rl-algo-impls_amd", "lib", "librai_amd.so")
    doc = {"workload": os.environ.get("C3_WORKLOAD", "ppo pong num_envs=1024/rank n_steps=128 (eager, RAI_GRAPHS=0)"),
           "lib_sha256": hashlib.sha256(open(libp, "rb").read()).hexdigest(),
           "optimizer_steps_per_update": STEPS,
           "bytes_per_optimizer_step": round(step_b),
           "bytes_per_update": round(step_b * STEPS + upd_b),
           "bytes_per_update_outside_steps": round(upd_b),
           "bytes_excluded_gemm_tuning_trials": round(dropped),
           "kernels": dict(top)}
    json.dump(doc, open(sys.argv[3], "w"), indent=1)
    print(f"per optimizer step {step_b / 1e6:.1f} MB, per update {(step_b * STEPS + upd_b) / 1e9:.2f} GB")
    for k, e in top[:12]:
        print(f"  {e['bytes_per_launch'] / 1e6:9.2f} MB x {e['dispatches']:5d}  {k[:90]}")


if __name__ == "__main__":
    main()
