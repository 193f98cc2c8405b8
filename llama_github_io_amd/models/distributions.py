"""Distributions and link functions (reference: ``h2o-core/src/main/java/hex/DistributionFactory.java``,
``hex/LinkFunctionFactory.java``). Vectorised in torch so they run on device inside the boosting loop.

Each distribution provides, per row: the pseudo-residual ``z = negHalfGradient(y, f)``, the Newton
leaf numerator/denominator terms ``gammaNum / gammaDenom``, the initial-prediction sums, deviance and
the inverse link.
"""
from __future__ import annotations

import math

import torch

LOG_CLAMP = 19.0  # LogExpUtil-style guard


def _exp(x):
    return torch.exp(torch.clamp(x, max=700.0))


class Distribution:
    name = "gaussian"
    link = "identity"

    def __init__(self, tweedie_power=1.5, quantile_alpha=0.5, huber_alpha=0.9):
        self.tweedie_power = tweedie_power
        self.quantile_alpha = quantile_alpha
        self.huber_alpha = huber_alpha
        self.huber_delta = 1.0

    # link functions
    def link_fn(self, mu):
        if self.link == "logit":
            return torch.log(mu / (1 - mu))
        if self.link == "log":
            return torch.log(mu)
        return mu

    def linkinv(self, f):
        if self.link == "logit":
            return torch.sigmoid(f)
        if self.link == "log":
            return _exp(f)
        return f

    def linkinv_scalar(self, f):
        if self.link == "logit":
            return 1.0 / (1.0 + math.exp(-f))
        if self.link == "log":
            return math.exp(f)
        return f

    def link_scalar(self, mu):
        if self.link == "logit":
            return math.log(mu / (1 - mu))
        if self.link == "log":
            return math.log(mu)
        return mu

    # boosting terms
    def neg_half_gradient(self, y, f):
        return y - self.linkinv(f)

    def gamma_num(self, w, y, z, f):
        return w * z

    def gamma_denom(self, w, y, z, f):
        return w

    def init_num(self, w, o, y):
        return w * (y - o)

    def init_denom(self, w, o, y):
        return w

    def init_f(self, y, w, offset=None, reduce=float):
        o = torch.zeros_like(y) if offset is None else offset
        num = reduce(self.init_num(w, o, y).double().sum().item())
        den = reduce(self.init_denom(w, o, y).double().sum().item())
        g = num / den if den != 0 else 0.0
        return self.gamma_to_f(g)

    def gamma_to_f(self, g):
        if self.name in ("poisson", "gamma", "tweedie"):
            return math.log(max(g, 1e-300))
        if self.name in ("bernoulli", "quasibinomial"):
            g = min(max(g, 1e-15), 1 - 1e-15)
            return math.log(g / (1 - g))
        return g

    def leaf_gamma(self, num, den):
        g = torch.where(den == 0, torch.zeros_like(num), num / torch.where(den == 0, torch.ones_like(den), den))
        if self.name in ("poisson", "gamma", "tweedie"):
            g = torch.where(den == 0, torch.zeros_like(g), torch.log(torch.clamp(g, min=1e-300)))
        return g

    def deviance(self, w, y, f):
        mu = self.linkinv(f)
        return w * (y - mu) ** 2


class Gaussian(Distribution):
    name, link = "gaussian", "identity"


class Bernoulli(Distribution):
    name, link = "bernoulli", "logit"

    def gamma_denom(self, w, y, z, f):
        ff = y - z
        return w * ff * (1 - ff)

    def init_f(self, y, w, offset=None, reduce=float):
        if offset is None:
            p = reduce((w * y).double().sum().item()) / max(reduce(w.double().sum().item()), 1e-300)
            p = min(max(p, 1e-15), 1 - 1e-15)
            return math.log(p / (1 - p))
        return super().init_f(y, w, offset, reduce)

    def deviance(self, w, y, f):
        p = torch.clamp(self.linkinv(f), 1e-15, 1 - 1e-15)
        return -2 * w * (y * torch.log(p) + (1 - y) * torch.log(1 - p))


class Quasibinomial(Bernoulli):
    name, link = "quasibinomial", "logit"

    def neg_half_gradient(self, y, f):
        ff = self.linkinv(f)
        return torch.where(ff == y, torch.zeros_like(ff),
                           torch.where(ff > 1, y / ff, torch.where(ff < 0, (1 - y) / (ff - 1), y - ff)))


class ModifiedHuber(Distribution):
    name, link = "modified_huber", "logit"

    def neg_half_gradient(self, y, f):
        s = 2 * y - 1
        yf = s * f
        return torch.where(yf < -1, 2 * s, torch.where(yf > 1, torch.zeros_like(f), -f * s * s))

    def gamma_num(self, w, y, z, f):
        s = 2 * y - 1
        yf = s * f
        return torch.where(yf < -1, w * 4 * s, torch.where(yf > 1, torch.zeros_like(f), w * 2 * s * (1 - yf)))

    def gamma_denom(self, w, y, z, f):
        s = 2 * y - 1
        yf = s * f
        return torch.where(yf < -1, -w * 4 * yf, torch.where(yf > 1, torch.zeros_like(f), w * (1 - yf) ** 2))

    def init_num(self, w, o, y):
        return torch.where(y == 1, w, torch.zeros_like(w))

    def init_denom(self, w, o, y):
        return torch.where(y == 1, torch.zeros_like(w), w)


class Multinomial(Distribution):
    name, link = "multinomial", "log"

    def gamma_denom(self, w, y, z, f):
        a = z.abs()
        return w * a * (1 - a)


class Poisson(Distribution):
    name, link = "poisson", "log"

    def gamma_num(self, w, y, z, f):
        return w * y

    def gamma_denom(self, w, y, z, f):
        return w * (y - z)

    def init_num(self, w, o, y):
        return w * y

    def init_denom(self, w, o, y):
        return w * _exp(o)

    def deviance(self, w, y, f):
        mu = _exp(f)
        t = torch.where(y > 0, y * torch.log(torch.where(y > 0, y, torch.ones_like(y)) / mu), torch.zeros_like(y))
        return 2 * w * (t - y + mu)


class Gamma(Distribution):
    name, link = "gamma", "log"

    def neg_half_gradient(self, y, f):
        return y * _exp(-f) - 1

    def gamma_num(self, w, y, z, f):
        return w * (z + 1)

    def init_num(self, w, o, y):
        return w * y * _exp(-o)

    def deviance(self, w, y, f):
        mu = _exp(f)
        return 2 * w * (torch.log(mu / y) + y / mu - 1)


class Tweedie(Distribution):
    name, link = "tweedie", "log"

    def neg_half_gradient(self, y, f):
        p = self.tweedie_power
        return y * _exp(f * (1 - p)) - _exp(f * (2 - p))

    def gamma_num(self, w, y, z, f):
        return w * y * _exp(f * (1 - self.tweedie_power))

    def gamma_denom(self, w, y, z, f):
        return w * _exp(f * (2 - self.tweedie_power))

    def init_num(self, w, o, y):
        return w * y * _exp(o * (1 - self.tweedie_power))

    def init_denom(self, w, o, y):
        return w * _exp(o * (2 - self.tweedie_power))

    def deviance(self, w, y, f):
        p = self.tweedie_power
        return 2 * w * (torch.pow(y, 2 - p) / ((1 - p) * (2 - p)) - y * _exp(f * (1 - p)) / (1 - p) + _exp(f * (2 - p)) / (2 - p))


class Laplace(Distribution):
    name, link = "laplace", "identity"

    def neg_half_gradient(self, y, f):
        return torch.where(f > y, torch.full_like(f, -0.5), torch.full_like(f, 0.5))

    def deviance(self, w, y, f):
        return w * (y - f).abs()


class Quantile(Distribution):
    name, link = "quantile", "identity"

    def neg_half_gradient(self, y, f):
        a = self.quantile_alpha
        return torch.where(y > f, torch.full_like(f, 0.5 * a), torch.full_like(f, 0.5 * (a - 1)))

    def deviance(self, w, y, f):
        a = self.quantile_alpha
        return torch.where(y > f, w * a * (y - f), w * (1 - a) * (f - y))


class Huber(Distribution):
    name, link = "huber", "identity"

    def neg_half_gradient(self, y, f):
        d = self.huber_delta
        r = y - f
        return torch.where(r.abs() <= d, r, torch.where(f >= y, torch.full_like(f, -d), torch.full_like(f, d)))

    def deviance(self, w, y, f):
        d = self.huber_delta
        r = (y - f).abs()
        return torch.where(r <= d, w * r * r, w * (2 * r - d) * d)


class Custom(Distribution):
    """``distribution="custom"`` with ``custom_distribution_func`` (DistributionFactory.CustomDistribution):
    gradient / init / gamma terms come from the uploaded CDistributionFunc (``udf.py``); leaves are the
    plain Newton ratio num/den (GBM.GammaPass.gamma applies no link for custom), the initial value is
    link(num/den) with the user's link."""
    name = "custom"

    def __init__(self, custom_distribution_func=None, **kw):
        super().__init__(**{k: v for k, v in kw.items() if k in ("tweedie_power", "quantile_alpha", "huber_alpha")})
        from ..udf import CustomDistributionFns
        if not custom_distribution_func:
            raise ValueError("distribution='custom' needs custom_distribution_func (h2o.upload_custom_distribution)")
        self.fns = CustomDistributionFns(custom_distribution_func)
        self.link = self.fns.link

    @staticmethod
    def _np(t):
        return t.detach().double().cpu().numpy()

    def _t(self, a, like):
        return torch.as_tensor(a, dtype=like.dtype, device=like.device)

    def linkinv(self, f):
        if self.link == "inverse":
            return 1.0 / f
        return super().linkinv(f)

    def neg_half_gradient(self, y, f):
        return self._t(self.fns.gradient(self._np(y), self._np(f)), f)

    def gamma_num(self, w, y, z, f):
        num, self._den = self.fns.gamma(self._np(w), self._np(y), self._np(z), self._np(f))
        return self._t(num, f)

    def gamma_denom(self, w, y, z, f):
        return self._t(self._den, f)

    def init_f(self, y, w, offset=None, reduce=float):
        o = torch.zeros_like(y) if offset is None else offset
        num, den = self.fns.init(self._np(w), self._np(o), self._np(y))
        g = reduce(float(num.sum())) / max(reduce(float(den.sum())), 1e-300)
        if self.link == "log":
            return math.log(max(g, 1e-300))
        if self.link == "logit":
            g = min(max(g, 1e-15), 1 - 1e-15)
            return math.log(g / (1 - g))
        if self.link == "inverse":
            return 1.0 / g
        return g

    def leaf_gamma(self, num, den):
        return torch.where(den == 0, torch.zeros_like(num), num / torch.where(den == 0, torch.ones_like(den), den))


_DISTS = {c.name: c for c in (Custom, Gaussian, Bernoulli, Quasibinomial, ModifiedHuber, Multinomial, Poisson, Gamma, Tweedie,
                              Laplace, Quantile, Huber)}
# quantile-type leaves (median / alpha-quantile of residuals per leaf)
ORDER_STAT_DISTS = ("laplace", "quantile", "huber")


def get_distribution(name: str, **kw) -> Distribution:
    name = name.lower()
    if name not in _DISTS:
        raise ValueError(f"unsupported distribution '{name}'")
    if name != "custom":
        kw.pop("custom_distribution_func", None)
    return _DISTS[name](**kw)
