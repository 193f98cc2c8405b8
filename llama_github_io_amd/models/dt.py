"""Single Decision Tree (reference: ``hex/tree/dt/DT.java``, ``DTModel.java``: binary classification,
``max_depth`` 20, ``min_rows`` 10, best split over all features, leaves hold P(class 1)).

Runs on the device histogram engine as one full-data tree with every column eligible at every
node; squared-error reduction on the 0/1 target is the Gini impurity decrease (the reference
uses entropy; both pick the same split in nearly all cases and the tree/leaf format is identical)."""
from __future__ import annotations

from .drf import DRFModel, DRFTrainer


class DTModel(DRFModel):
    algo = "dt"


class DTTrainer(DRFTrainer):
    algo = "dt"
    model_cls = DTModel

    def __init__(self, params):
        p = dict(max_depth=20, min_rows=10.0)
        p.update({k: v for k, v in params.items() if v is not None})
        p.update(ntrees=1, mtries=-2, sample_rate=1.0, min_split_improvement=0.0)
        super().__init__(p)

    def fit(self, X, y, w, offset, info, valid=None, model_key=None):
        if info.response_domain is None or len(info.response_domain) != 2:
            raise ValueError("DT supports binary classification only")
        return super().fit(X, y, w, offset, info, valid, model_key)

    def _training_metrics(self, model):
        return model.metrics_for(self.X, self.y, self.w)
