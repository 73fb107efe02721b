"""caldera-mi355x: MI355X-native CALDERA/LPLR weight decomposition.

Drop-in API (same names as the reference): `src.caldera.decomposition.alg.caldera`,
`src.caldera.utils.dataclasses.CalderaParams`, `src.caldera.utils.quantization.QuantizerFactory`.
Batched / multi-GPU entry points: `api.caldera_batch`, `sharding.decompose_sharded`.
"""
__version__ = "0.1.0"
