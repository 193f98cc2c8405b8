"""Munging transforms of an :class:`h2o.assembly.H2OAssembly` (reference ``h2o-py/h2o/transforms``)."""
from .preprocessing import H2OBinaryOp, H2OColOp, H2OColSelect, H2OScaler  # noqa: F401
from .transform_base import H2OTransformer  # noqa: F401
