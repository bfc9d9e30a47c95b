"""Data-parallel host logic on CPU with the gloo backend, world_size=2."""
import multiprocessing as mp
import socket

import numpy as np


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_global_advantage_moments_world2():
    import dp_worker

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=dp_worker.moments_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs = dict(res)
    for case in range(3):  # one column; K=3 columns; weighted advantage (after scaling)
        o0, ref0 = (np.array(x) for x in outs[0][case])
        o1, _ = (np.array(x) for x in outs[1][case])
        np.testing.assert_array_equal(o0, o1)  # identical on every rank
        np.testing.assert_allclose(o0, ref0, rtol=1e-5, atol=1e-6)


def test_dp_batch_rules_world2():
    import dp_worker

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=dp_worker.batch_rule_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in (0, 1):
        out = res[rank]
        assert out[("per-rank", 256)][:2] == (256, 512)
        assert out[("global", 256)][:2] == (128, 256)  # B / R rows per rank
        assert "not divisible" in out[("global", 255)]
        assert out["repeat"] == [(128, 256), (128, 256), (256, 512), (128, 256)]
    assert res[0][("global", 256)][2] == res[1][("global", 256)][2]  # identical weights after the broadcast


def test_replicated_update_rollout_assembly_world2():
    """update_mode='replicated': every rank keeps the YAML minibatch (the single-process update runs on
    each), 'per-rank' batches are rejected, a CPU trainer's 'auto' keeps the exchange rule; the whole
    env group's rollout is rank 0's envs then rank 1's (bitwise), identical on both ranks, and both
    ranks draw the same shuffle keys (derived from rank 0's)."""
    import dp_worker

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=dp_worker.replicated_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in (0, 1):
        out = res[rank]
        assert out["sizes"] == (256, 256, "replicated")
        assert "dp_batch='global'" in out["per_rank"]
        assert out["auto_cpu"] == (128, "exchange")
        assert out["total_steps"] == 5 * 6
        for k, v in out["gathered"].items():
            want = np.concatenate([res[0]["local"][k], res[1]["local"][k]], axis=1)
            np.testing.assert_array_equal(v, want, err_msg=k)
    assert res[0]["params"] == res[1]["params"]
    assert res[0]["keys"] == res[1]["keys"] and len(set(res[0]["keys"])) == 3
