"""sdf_nmpc_amd -- MI355X-native evaluator for the neural-SDF NMPC hot path of ntnu-arl/sdf-nmpc.

Hot path (BASELINE.json ``north_star``): NeuralDF forward + position-Jacobian and the per-stage
dynamics / cost / constraint linearisation of the SQP-RTI loop, batched over (MPC instance x shooting
node) in hand-written HIP kernels for gfx950, behind a C ABI (``include/sdfnmpc.h``,
``include/sdf_l4c.h``).  Python here is the host-side mirror of the reference's ``controller.py`` /
``ocp.py`` API; it never computes the hot path itself.
"""
__version__ = "0.1.0"
