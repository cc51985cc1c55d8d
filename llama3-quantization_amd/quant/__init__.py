"""MI355X-native build of the reference ``quant`` package (SilviaUvA/LLaMA3-Quantization).

Same module / class names as the reference: ``quant.quantizer.UniformAffineQuantizer``,
``quant.int_linear.QuantLinear``, ``quant.int_matmul.QuantMatMul``, ``quant.omni_norm``,
``quant.utils``.  Arithmetic runs in hand-written gfx950 HIP kernels behind the C ABI of
``libqlin_gfx950.so`` (``quant.qlin``).
"""
