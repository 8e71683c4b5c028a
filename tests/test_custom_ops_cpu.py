"""The torch.ops.adaptseg op surface (adaptsegnet_amd/ops.py), host-side checks (no GPU).

Every launch of the package is a registered custom operator with a CUDA (= HIP) kernel and
a fake kernel; none has a CPU kernel, so calling one on CPU tensors fails loudly; the fake
kernels let FakeTensorMode trace the tensor-level API (shape propagation only, nothing runs).
"""
import pytest
import torch


def test_every_op_is_registered_with_cuda_and_fake_kernels():
    from adaptsegnet_amd import ops
    assert len(ops.NAMES) >= 30
    for name in ops.NAMES:
        op = getattr(torch.ops.adaptseg, name).default
        assert torch._C._dispatch_has_kernel_for_dispatch_key(op.name(), "CUDA"), name
        assert not torch._C._dispatch_has_kernel_for_dispatch_key(op.name(), "CPU"), name
        # every op is an out-variant: mutable outputs, no returns
        schema = op._schema
        assert len(schema.returns) == 0, name
        assert any(a.alias_info is not None and a.alias_info.is_write for a in schema.arguments), name
        assert getattr(ops.OPS, name) is op


def test_cpu_tensors_raise():
    from adaptsegnet_amd import kernels as K
    with pytest.raises(NotImplementedError, match="adaptseg::softmax_fwd"):
        K.softmax_fwd(torch.zeros(2, 4, 4, 19))
    g = K.ConvGeom(8, 16, 3, 3, 1, (1,), (1,))
    with pytest.raises(NotImplementedError, match="adaptseg::conv2d_fwd"):
        K.conv_fwd(g, torch.zeros(1, 6, 6, 8), 1, 6, 6, [torch.zeros(16, 8, 3, 3)])


def test_fake_tensor_tracing_of_the_tensor_api():
    from torch._subclasses.fake_tensor import FakeTensorMode
    from adaptsegnet_amd import kernels as K
    with FakeTensorMode():
        x = torch.empty(2, 32, 40, 64, device="cuda")
        g = K.ConvGeom(64, 128, 3, 3, 1, (2,), (2,))
        w = torch.empty(128, 64, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)
        y = K.conv_fwd(g, x, 2, 32, 40, [w])
        assert y.shape == (2, 32, 40, 128)
        dx = K.conv_dgrad(g, y, 2, 32, 40, [w])
        assert dx.shape == x.shape
        z, mean, invstd = K.bn_fwd_train(y, torch.ones(128, device="cuda"), torch.zeros(128, device="cuda"),
                                         None, None, 0.1, 1e-5)
        assert z.shape == y.shape and mean.shape == (128,)
        u = K.upsample_fwd(torch.empty(2, 8, 10, 19, device="cuda"), 64, 80)
        assert u.shape == (2, 64, 80, 19)
        assert K.ce_fwd(u, torch.empty(2, 64, 80, dtype=torch.int64, device="cuda")).shape == (2,)


def test_pack_cache_keeps_one_finalizer_per_weight():
    """kernels._PackCache: clear_weight_packs() then reusing a weight does not register a second
    weakref finalizer on it, and dropping the weight removes both its pack dict and
    its finalizer."""
    import gc
    from adaptsegnet_amd import kernels as K
    t = torch.zeros(8)
    wid = id(t)
    K._PACKS.track(t)["k"] = 1
    K.clear_weight_packs()
    assert wid not in K._PACKS.entries
    for _ in range(3):
        K._PACKS.track(t)
        K.clear_weight_packs()
    K._PACKS.track(t)
    live = [f for f in weakref_finalizers_of(t)]
    assert len(live) == 1, live
    assert K._PACKS.finalizers[wid].alive
    del t
    gc.collect()
    assert wid not in K._PACKS.entries and wid not in K._PACKS.finalizers


def weakref_finalizers_of(obj):
    import weakref
    return [f for f in list(weakref.finalize._registry) if f.peek() and f.peek()[0] is obj]
