"""In-process tree inspection (reference ``h2o-py/h2o/tree``): :class:`H2OTree` and its node classes."""
from .tree import H2OLeafNode, H2ONode, H2OSplitNode, H2OTree  # noqa: F401
