"""Diagnostic (GPU): where the Moore block-1 unified learner's tables leave the CPU
restatement -- tiled vs accumulator path, raster vs workgroup shapes.  Prints per case
the first table mismatch (missing / extra keys decoded as rank | bx | by)."""
import os
import sys
import traceback

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))


def run(tag, tiled_env, **kw):
    if tiled_env is None:
        os.environ.pop("FFM_TILED", None)
    else:
        os.environ["FFM_TILED"] = tiled_env
    import test_gpu_learn as T
    try:
        T._philox_compare(**kw)
        print(f"{tag}: OK", flush=True)
    except AssertionError as e:
        print(f"{tag}: FAIL {str(e).splitlines()[0][:200]}", flush=True)
    except Exception:
        print(f"{tag}: ERROR", flush=True)
        traceback.print_exc()


def dump(path, T_=3, mode="critic_only", N=600, tiled_env=None):
    """The GPU learner's state and V keys after T_ steps (analysed against the CPU side apart)."""
    if tiled_env is None:
        os.environ.pop("FFM_TILED", None)
    else:
        os.environ["FFM_TILED"] = tiled_env
    import test_gpu_learn as T
    from ffm_amd.data import make_room, l1_sff
    m = make_room(64, 64)
    s = l1_sff(m).astype(np.float32)
    p = {"epsilon": 0.1, "block_size": 1, "neighborhood": "moore"}
    L = T._learner(m, s, "unified", n_envs=16, n_agents=N, agent_capacity=N, mode=mode, params=p, rng="philox",
                   seed=4, auto_reset=True, max_steps=20, env_base=0)
    L.reset()
    out = {}
    for t in range(1, T_ + 1):
        L.step(1)
        gp, gc, gd = L.get_state()
        k, v = L.export_table("V")
        out[f"pos{t}"], out[f"cnt{t}"], out[f"vk{t}"], out[f"vv{t}"] = gp, gc, k, np.asarray(v)
    np.savez(path, **out)
    L.close()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "dump":
        os.makedirs("gpurun_out", exist_ok=True)
        dump("gpurun_out/moore_critic_dump.npz")
        return
    p = {"epsilon": 0.1, "block_size": 1, "neighborhood": "moore"}
    base = dict(variant="unified", params=p, H=64, W=64, N=600, E=16, T=30, max_steps=20, seed=4)
    for mode in ("critic_only", "actor_only"):
        run(f"{mode} tiled", None, mode=mode, **base)
        run(f"{mode} acc", "0", mode=mode, **base)
    for T_ in (1, 2, 3, 5, 10):
        run(f"critic tiled T={T_}", None, mode="critic_only", **dict(base, T=T_))
        run(f"critic acc T={T_}", "0", mode="critic_only", **dict(base, T=T_))
    run("critic 200 agents (256-lane)", None, mode="critic_only", **dict(base, N=200))
    run("critic neumann tiled", None, mode="critic_only", **dict(base, params={"epsilon": 0.1, "block_size": 1}))


if __name__ == "__main__":
    main()
