"""PINN path of the reference (pinn_kalman/): FlowNet + PressureNet and the
Navier-Stokes residual, on the gfx950 correlation / grid_sample kernels."""
