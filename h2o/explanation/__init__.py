"""h2o.explanation — model explanations (reference: ``h2o-py/h2o/explanation/_explain.py``).

Every function computes its table on the engine (variable importances, model correlations, TreeSHAP
contributions, partial dependence / ICE, residuals, scoring history, Pareto front) and draws it with
matplotlib when that is importable (Agg backend, no display needed). Each returns an
:class:`Explanation`: ``.data`` is the pandas table behind the plot, ``.figure()`` the matplotlib
figure (``None`` without matplotlib). ``explain`` / ``explain_row`` bundle them like the reference's
``H2OExplanation`` (a dict of sections).
"""
from __future__ import annotations

from ._explain import (Explanation, disparate_analysis, explain, explain_row, ice_plot, learning_curve_plot,  # noqa: F401
                       model_correlation, model_correlation_heatmap, pareto_front, pd_multi_plot, pd_plot,
                       residual_analysis_plot, shap_explain_row_plot, shap_summary_plot, varimp, varimp_heatmap,
                       register_explain_methods)

__all__ = ["explain", "explain_row", "varimp_heatmap", "model_correlation_heatmap", "pd_multi_plot", "varimp",
           "model_correlation", "pareto_front", "shap_summary_plot", "shap_explain_row_plot", "pd_plot", "ice_plot",
           "residual_analysis_plot", "learning_curve_plot", "disparate_analysis"]
