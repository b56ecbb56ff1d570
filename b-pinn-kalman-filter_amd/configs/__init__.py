"""ml_collections-style configs (reference: configs/**, main.py:31).

`get_config()` in each module returns a ConfigDict with the reference's sections
(training / sampling / eval / data / model / optim, + inverse / kf for PINN).
"""
