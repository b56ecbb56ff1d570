"""Host logic of the PINN step factory: graph=True builds the hipGraph step object
(losses._PinnGraphStep: captured on its first call, on a HIP device), the default builds the
eager step; both are callables with the reference's step_fn(state, operator, batch) contract."""
import pytest  # noqa: F401


def test_pinn_step_factory_forms():
    import losses
    from configs.pinn import pinn_pde
    c = pinn_pde.get_config()
    g = losses.get_pinn_step_fn(c, train=True, optimize_fn=losses.optimization_manager(c),
                                graph=True)
    assert isinstance(g, losses._PinnGraphStep) and g.graph is None  # nothing captured yet
    assert callable(losses.get_pinn_step_fn(c, train=True,
                                            optimize_fn=losses.optimization_manager(c)))
    # evaluation (train=False) has no graph form: the eager function is returned
    ev = losses.get_pinn_step_fn(c, train=False, optimize_fn=losses.optimization_manager(c),
                                 graph=True)
    assert not isinstance(ev, losses._PinnGraphStep)


def test_mask_operator_is_the_keep_shape_inpainting_product():
    import torch
    import losses
    m = (torch.rand(2, 1, 4, 4) > 0.5).float()
    op = losses._MaskOperator(m)
    x = torch.randn(2, 1, 4, 4)
    assert torch.equal(op(x), m * x) and torch.equal(op(x, invert=True), (1 - m) * x)
