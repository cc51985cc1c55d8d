"""Module-level helpers of the reference quant/utils.py that the hot path uses
(``set_quant_state`` :138, ``register_scales_and_zeros`` :39, ``smooth_and_quant_inplace`` :112 without
LET), plus ``pack_quant_linears`` — the MI355X real-quant pass (quant/omniquant.py:315-335)."""
import torch

from .int_linear import QuantLinear
from .int_matmul import QuantMatMul


def register_scales_and_zeros(model):
    for name, module in model.named_modules():
        if isinstance(module, QuantLinear):
            module.weight_quantizer.register_scales_and_zeros()


@torch.no_grad()
def smooth_and_quant_inplace(model, args=None, isllama=True):
    """RTN weight fake-quant in place (quant/utils.py:111-136 with ``args.let`` False).

    LET (learnable equivalent transformation) is a calibration-time rewrite outside the hot path
     and is rejected rather than silently skipped."""
    if args is not None and getattr(args, "let", False):
        raise NotImplementedError("LET smoothing is out of scope for the MI355X hot path")
    for name, module in model.named_modules():
        if isinstance(module, QuantLinear):
            module.weight = module.weight_quantizer(module.weight)
            module.use_temporary_parameter = False


def set_quant_state(self, weight_quant: bool = False, act_quant: bool = False):
    self.use_weight_quant = weight_quant
    self.use_act_quant = act_quant
    for m in self.modules():
        if isinstance(m, (QuantLinear, QuantMatMul)):
            m.set_quant_state(weight_quant, act_quant)


@torch.no_grad()
def pack_quant_linears(model, keep_weight=False):
    """Pack every registered QuantLinear of ``model`` into the gfx950 layout (the ``--real_quant``
    step).  Returns the number of packed modules."""
    n = 0
    for name, module in model.named_modules():
        if isinstance(module, QuantLinear) and not module.packed and \
                module.weight_quantizer.n_bits < 16:
            module.pack(keep_weight=keep_weight)
            n += 1
    return n
