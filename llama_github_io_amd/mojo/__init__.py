"""MOJO export / import (reference: ``h2o-genmodel`` — ``AbstractMojoWriter``, ``ModelMojoReader``,
``SharedTreeMojoModel``, ``GlmMojoModel``, ``KMeansMojoModel``, ``IsolationForestMojoModel``)."""
