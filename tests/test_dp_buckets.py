"""GradBuckets (dp_buckets.py) host logic on CPU: bucket bounds of the NatureCNN policy, trigger
order, every bucket reduced exactly once per step, the 1/world scale."""
import torch

from rl_algo_impls_amd.dp_buckets import GradBuckets, nature_cnn_buckets, notify_grad_written
from rl_algo_impls_amd.envs import SyntheticVecEnv
from rl_algo_impls_amd.optim import FlatParams
from rl_algo_impls_amd.policy import ActorCritic


def test_nature_cnn_bucket_layout_and_launch_order():
    torch.manual_seed(0)
    pol = ActorCritic(SyntheticVecEnv(2, "pong", seed=0), activation_fn="relu")
    flat = FlatParams(pol, torch.device("cpu"))
    bounds, triggers = nature_cnn_buckets(pol, flat)
    fc_w = pol.network._feature_extractor.feature_extractor.fc[1].weight
    names = [n for n, _ in pol.named_parameters()]
    k = names.index("network._feature_extractor.feature_extractor.fc.1.weight")
    assert bounds == [0, flat.offsets[k], flat.P]
    assert triggers == {id(fc_w): 1}
    # conv bucket 0.31 MB, fc + heads bucket 6.43 MB (6,750,876 B in total)
    assert 4 * flat.P == 6750876
    assert 4 * bounds[1] == 4 * (8192 + 32 + 32768 + 64 + 36864 + 64)

    order = []

    def allreduce(v):
        order.append((v.data_ptr() - flat.grad.data_ptr()) // 4)
        v.add_(1.0)  # "sum" with a second rank holding ones

    gb = GradBuckets(flat, bounds, triggers, allreduce, torch.device("cpu"))
    assert not gb.overlap  # CPU: no side stream; buckets are reduced at finish()
    flat.grad.zero_()
    gb.begin()
    notify_grad_written(fc_w)
    gb.finish(scale=0.5)
    assert order == [bounds[1], 0]  # later layers first, each bucket once
    assert torch.equal(flat.grad, torch.full_like(flat.grad, 0.5))


def test_no_bucket_layout_for_mlp_policies():
    torch.manual_seed(0)
    pol = ActorCritic(SyntheticVecEnv(2, "cartpole", seed=0))
    assert nature_cnn_buckets(pol, FlatParams(pol, torch.device("cpu"))) is None


def test_trigger_hook_fires_from_another_thread():
    """Autograd runs CUDA backward nodes on its per-device worker thread, not on the thread that
    armed the buckets: the trigger hook is process-wide (a thread-local hook never fired there and
    every bucket waited for finish())."""
    import threading

    from rl_algo_impls_amd import dp_buckets

    seen = []
    p = torch.zeros(3)
    dp_buckets._hooks.cb = seen.append
    try:
        th = threading.Thread(target=notify_grad_written, args=(p,))
        th.start()
        th.join()
    finally:
        dp_buckets._hooks.cb = None
    assert len(seen) == 1 and seen[0] is p
    notify_grad_written(p)  # disarmed: nothing
    assert len(seen) == 1


def test_deferred_weight_gradient_accumulates():
    """cnn_ops.direct_grads: the convolution weight gradients queued during the backward are added
    by one multi-tensor add at the context's exit, in place into the (flat-buffer) .grad views; a
    backward that runs after the context has closed adds its own at once; an exception inside the
    context drops the queue."""
    from rl_algo_impls_amd import cnn_ops

    w1, w2 = torch.zeros(2, 3, requires_grad=True), torch.zeros(4, requires_grad=True)
    w1.grad, w2.grad = torch.ones(2, 3), torch.ones(4)
    with cnn_ops.direct_grads(True):
        pending = cnn_ops._state.pending
        pending.add(w1, torch.full((2, 3), 2.0))
        pending.add(w2, torch.full((4,), 3.0))
        assert torch.equal(w1.grad, torch.ones(2, 3))  # nothing added before the exit
    assert torch.equal(w1.grad, torch.full((2, 3), 3.0)) and torch.equal(w2.grad, torch.full((4,), 4.0))
    pending.add(w2, torch.full((4,), 1.0))  # closed: immediate
    assert torch.equal(w2.grad, torch.full((4,), 5.0))
    try:
        with cnn_ops.direct_grads(True):
            cnn_ops._state.pending.add(w2, torch.full((4,), 100.0))
            raise RuntimeError("backward failed")
    except RuntimeError:
        pass
    assert torch.equal(w2.grad, torch.full((4,), 5.0))
    assert getattr(cnn_ops._state, "pending", None) is None and not getattr(cnn_ops._state, "direct", False)
