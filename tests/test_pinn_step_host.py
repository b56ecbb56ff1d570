"""Host-side contract of the PINN step factory (no GPU): the hipGraph replay form was
withdrawn in round 3, so asking for it must fail loudly instead of
silently returning the eager step."""
import pytest


def test_pinn_step_graph_is_refused():
    import losses
    from configs.pinn import pinn_pde
    c = pinn_pde.get_config()
    with pytest.raises(NotImplementedError, match="graph=True"):
        losses.get_pinn_step_fn(c, train=True, optimize_fn=losses.optimization_manager(c),
                                graph=True)
    # the default (eager) form still builds
    assert callable(losses.get_pinn_step_fn(c, train=True,
                                            optimize_fn=losses.optimization_manager(c)))
