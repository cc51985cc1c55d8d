"""MI355X build of the reference ``models`` per-layer dispatch (models/int_llama_layer.py,
models/int_opt_layer.py): every linear is a ``quant.int_linear.QuantLinear``."""
