"""Base class of the assembly transforms (reference ``h2o-py/h2o/transforms/transform_base.py``)."""
from __future__ import annotations


class TransformAttributeError(AttributeError):
    def __init__(self, obj, method):
        super().__init__(f"No {method} method for {obj.__class__.__name__}")


class H2OTransformer:
    """fit / transform / fit_transform / inverse_transform / to_rest; ``to_rest(args)`` joins the step's wire
    fields with ``__`` (name, class, Rapids AST over the placeholder frame ``dummy``, inplace, new names)."""

    parms: dict = {}

    def fit(self, X, y=None, **params):
        raise TransformAttributeError(self, "fit")

    def transform(self, X, y=None, **params):
        raise TransformAttributeError(self, "transform")

    def inverse_transform(self, X, y=None, **params):
        raise TransformAttributeError(self, "inverse_transform")

    def export(self, X, y, **params):
        raise TransformAttributeError(self, "export")

    def fit_transform(self, X, y=None, **params):
        return self.fit(X, y, **params).transform(X, **params)

    def get_params(self, deep=True):
        out = {}
        for key, value in self.parms.items():
            if deep and isinstance(value, H2OTransformer):
                out.update((key + "__" + k, v) for k, v in value.get_params().items())
            out[key] = value
        return out

    def set_params(self, **params):
        self.parms.update(params)
        return self

    def to_rest(self, args):
        return "__".join(str(a) for a in args)
