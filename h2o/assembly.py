"""H2OAssembly: several frame munging steps as one pipeline, exportable as a per-row Java POJO (reference
``h2o-py/h2o/assembly.py``; engine ``llama_github_io_amd/assembly.py``)."""
from __future__ import annotations

import os
import uuid

from llama_github_io_amd import assembly as _asm
from llama_github_io_amd.frame import H2OFrame

from .transforms.transform_base import H2OTransformer


class H2OAssembly:
    """``H2OAssembly(steps=[(name, transform), ...])``; ``fit(frame)`` runs the steps and returns the munged frame,
    ``to_pojo`` writes the GenMunger Java source of the fitted pipeline."""

    divide = H2OFrame.__truediv__
    plus = H2OFrame.__add__
    multiply = H2OFrame.__mul__
    minus = H2OFrame.__sub__
    less_than = H2OFrame.__lt__
    less_than_equal = H2OFrame.__le__
    equal_equal = H2OFrame.__eq__
    not_equal = H2OFrame.__ne__
    greater_than = H2OFrame.__gt__
    greater_than_equal = H2OFrame.__ge__

    def __init__(self, steps):
        for step in steps:
            if not (isinstance(step, tuple) and len(step) == 2 and isinstance(step[0], str)
                    and isinstance(step[1], H2OTransformer)):
                raise TypeError("steps must be a list of (name, H2OTransformer) tuples")
        self.id = None
        self.steps = steps
        self.fuzed = []
        self.in_colnames = None
        self.out_colnames = None
        self._assembly = None

    @property
    def names(self):
        return list(zip(*self.steps))[0][:-1]

    def fit(self, fr):
        """Run the steps on ``fr`` (through the engine's Assembly, as POST /99/Assembly does)."""
        if not isinstance(fr, H2OFrame):
            raise TypeError("fit needs an H2OFrame")
        steps = [st.to_rest(name).replace('"', "'") for name, st in self.steps]
        self._assembly, out = _asm.fit_rest(steps, fr)
        self.id = self._assembly.key
        return out

    def to_pojo(self, pojo_name="", path="", get_jar=True):
        if self._assembly is None:
            raise ValueError("fit the assembly before exporting it")
        if pojo_name == "":
            pojo_name = "AssemblyPOJO_" + str(uuid.uuid4())
        java = self._assembly.to_java(pojo_name)
        if path == "":
            print(java)
        else:
            with open(os.path.join(path, pojo_name + ".java"), "w", encoding="utf-8") as f:
                f.write(java)
        return java

    def download_mojo(self, file_name="", path="."):
        raise NotImplementedError("MOJO 2 munging pipelines need the mojo2-runtime library, which this engine does "
                                  "not ship; use to_pojo")
