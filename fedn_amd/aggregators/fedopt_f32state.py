"""FedOpt with float32 server state — an opt-in variant of the fedopt plug-in (SURVEY.md §7 step 5:
"an fp32-state mode validated to <= 1e-6 relative against the oracle").

The reference's FedOpt (fedopt.py:151-258) keeps ``v`` in float64 from the first round
(``np.ones(...) * tau**2``, numpyhelper.py:129-142), and with it ``m`` and the returned model
(float32 updates promote against a float64 global model). For a float32 model that doubles the
bytes of every state stream: a steady-state round moves P*(4K + 48) bytes. Here, for every tensor
group whose global model is float32, ``m``, ``v`` and the new model are STORED in float32 and
read back widened exactly: P*(4K + 24) bytes. The arithmetic of each round is the reference's on
the values it is given (the same fused kernel, fa_fedopt_step_ex with state_dtype F32): every
stored value is the reference step's float64 result rounded once to float32, the pseudo-gradient
is float32 as numpy computes it for a float32 model, and the returned model is float32.

Parity: per round, m / v / model equal float32(reference step on the same stored inputs)
bit-for-bit; over a session, the model stays within 1e-6 relative of the reference's float64
session (tests/test_gpu_fedopt_f32state.py).

A separate module (FEDn selects aggregators by module name, aggregatorbase.py:44-62) because
FEDn's ``Parameters.validate`` refuses unknown keys (fedopt.py:123-137): the hyper-parameters are
the fedopt plug-in's. Install with a shim ``fedn/network/combiner/aggregators/fedopt_f32state.py``
(INTEGRATION.md).
"""
from . import fedopt


class Aggregator(fedopt.Aggregator):
    """FedAdam / FedYogi / FedAdaGrad with float32 server state for float32 models."""

    fp32_state = True

    def __init__(self, update_handler, device=None, devices=None):
        super().__init__(update_handler, device=device, devices=devices)
        self.name = "fedopt_f32state"
