"""Fold iterators over H2OFrames for sklearn-style cross validation (reference: h2o-py/h2o/cross_validation.py):
each iteration yields (train mask, test mask) frames of 0 / 1."""


class H2OPartitionIterator:
    def __init__(self, n):
        if abs(n - int(n)) >= 1e-15:
            raise ValueError("n must be an integer")
        self.n = int(n)
        self.masks = None

    def __iter__(self):
        for test in self._test_masks():
            yield 1 - test, test

    def _test_masks(self):
        raise NotImplementedError()


class _Folds(H2OPartitionIterator):
    def __init__(self, src, n_folds, seed, how):
        super().__init__(src.nrows)
        self.n_folds, self.seed, self._src, self._how = n_folds, seed, src, how
        self.fold_assignments = None

    def __len__(self):
        return self.n_folds

    def _test_masks(self):
        if self.fold_assignments is None:
            if self._src is None:
                raise ValueError("No frame available for computing folds.")
            self.fold_assignments = getattr(self._src, self._how)(self.n_folds, self.seed)
            self._src = None
        if self.masks is None:
            self.masks = [self.fold_assignments == i for i in range(self.n_folds)]
        return self.masks


class H2OKFold(_Folds):
    """Random k folds of the rows of ``fr`` (H2OFrame.kfold_column)."""

    def __init__(self, fr, n_folds=3, seed=-1):
        super().__init__(fr, n_folds, seed, "kfold_column")


class H2OStratifiedKFold(_Folds):
    """Folds stratified by the response column ``y`` (H2OFrame.stratified_kfold_column)."""

    def __init__(self, y, n_folds=3, seed=-1):
        super().__init__(y, n_folds, seed, "stratified_kfold_column")
