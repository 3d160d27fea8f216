"""Diffusion samplers for the Stable Diffusion pipeline (models/sd.py): every scheduler name the
reference's diffusers backend accepts (`backend/python/diffusers/backend.py:74-143`, the A1111
naming: ddim, pndm, heun, unipc, euler, euler_a, lms, dpm_2, dpm_2_a, dpmpp_2m, dpmpp_sde,
dpmpp_2m_sde, each with a `k_` Karras-sigma variant).

Two families over the same trained noise schedule (alphas_cumprod from scheduler_config.json):
  * timestep-space: DDIM (eta 0) and PNDM's PLMS (linear multistep on eps with the pseudo
    Runge-Kutta warm-up replaced by lower orders, diffusers `skip_prk_steps`);
  * sigma-space (k-diffusion formulation, x = x0 + sigma * eps): the model is wrapped as a
    denoiser D(x, sigma) (input scaled by 1/sqrt(sigma^2 + 1), sigma mapped to a fractional
    training timestep by log-sigma interpolation, eps / v-prediction converted to x0), and the
    samplers are ODE / SDE integrators over a descending sigma list -- linspace-in-timestep
    sigmas, or Karras sigmas (rho = 7) for the `k_` names.
diffusers is not installed here, so the samplers are checked against the analytic denoiser of
Gaussian data (tests/test_schedulers.py: every sampler must map the prior onto N(mu, s^2)).
"""
from __future__ import annotations

import math
from typing import Callable, List, Optional, Sequence

import torch

NAMES = ("ddim", "pndm", "heun", "unipc", "euler", "euler_a", "lms", "dpm_2", "dpm_2_a", "dpmpp_2m", "dpmpp_sde",
         "dpmpp_2m_sde")


def parse_name(name: str):
    """-> (base name, karras).  Unknown names raise, as the reference's get_scheduler does."""
    n = (name or "ddim").lower()
    karras = n.startswith("k_")
    base = n[2:] if karras else n
    if base not in NAMES:
        raise ValueError(f"Invalid scheduler '{name}'")
    return base, karras


def train_alphas_cumprod(c: dict) -> torch.Tensor:
    n = int(c.get("num_train_timesteps", 1000))
    b0, b1 = float(c.get("beta_start", 0.00085)), float(c.get("beta_end", 0.012))
    if c.get("beta_schedule", "scaled_linear") == "linear":
        betas = torch.linspace(b0, b1, n, dtype=torch.float64)
    else:
        betas = torch.linspace(b0 ** 0.5, b1 ** 0.5, n, dtype=torch.float64) ** 2
    return torch.cumprod(1.0 - betas, 0)


def karras_sigmas(n: int, smin: float, smax: float, rho: float = 7.0) -> List[float]:
    r = torch.linspace(0, 1, n, dtype=torch.float64)
    return ((smax ** (1 / rho) + r * (smin ** (1 / rho) - smax ** (1 / rho))) ** rho).tolist()


class SigmaSchedule:
    """The trained sigmas and the sigma <-> fractional-timestep map (k-diffusion DiscreteSchedule)."""

    def __init__(self, ac: torch.Tensor):
        self.sigmas = ((1 - ac) / ac) ** 0.5            # ascending in t
        self.log_sigmas = self.sigmas.log()

    def sigma_to_t(self, sigma: float) -> float:
        ls = math.log(max(sigma, 1e-12))
        d = ls - self.log_sigmas
        low = int((d >= 0).cumsum(0).argmax().clamp(max=len(self.log_sigmas) - 2))
        lo, hi = float(self.log_sigmas[low]), float(self.log_sigmas[low + 1])
        w = min(max((lo - ls) / (lo - hi), 0.0), 1.0)
        return (1 - w) * low + w * (low + 1)

    def t_to_sigma(self, t: float) -> float:
        lo = int(math.floor(t))
        hi = min(lo + 1, len(self.sigmas) - 1)
        w = t - lo
        return math.exp((1 - w) * float(self.log_sigmas[lo]) + w * float(self.log_sigmas[hi]))


def timestep_grid(n_train: int, steps: int, spacing: str, offset: int) -> List[float]:
    """Descending inference timesteps (diffusers `timestep_spacing`)."""
    if spacing == "leading":
        r = n_train // steps
        return [float(i * r + offset) for i in range(steps)][::-1]
    if spacing == "trailing":
        r = n_train / steps
        return [float(round(n_train - i * r) - 1) for i in range(steps)]
    return torch.linspace(0, n_train - 1, steps, dtype=torch.float64).flip(0).tolist()   # linspace


class KSampler:
    """Sigma-space samplers.  `denoise(x, sigma) -> x0` is the wrapped model."""

    def __init__(self, c: dict, name: str):
        self.base, self.karras = parse_name(name)
        self.ac = train_alphas_cumprod(c)
        self.sched = SigmaSchedule(self.ac)
        self.spacing = c.get("timestep_spacing", "linspace")
        self.offset = int(c.get("steps_offset", 0))

    def sigmas(self, steps: int) -> List[float]:
        if self.karras:
            s = karras_sigmas(steps, float(self.sched.sigmas[0]), float(self.sched.sigmas[-1]))
        else:
            n = len(self.ac)
            s = [self.sched.t_to_sigma(min(t, n - 1)) for t in timestep_grid(n, steps, self.spacing, self.offset)]
        return s + [0.0]

    @staticmethod
    def _ancestral(s_from: float, s_to: float, eta: float = 1.0):
        if s_to == 0:
            return 0.0, 0.0
        up = min(s_to, eta * math.sqrt(max(s_to ** 2 * (s_from ** 2 - s_to ** 2) / s_from ** 2, 0.0)))
        return math.sqrt(max(s_to ** 2 - up ** 2, 0.0)), up

    def sample(self, denoise: Callable[[torch.Tensor, float], torch.Tensor], x: torch.Tensor, sigmas: Sequence[float],
               gen: Optional[torch.Generator] = None) -> torch.Tensor:
        """x already carries sigmas[0] of noise; returns the x0 sample."""
        noise = lambda: torch.randn(x.shape, generator=gen).to(x.device, x.dtype)  # noqa: E731
        b, n = self.base, len(sigmas) - 1
        old_den, h_last, ds, pc = None, None, [], None
        for i in range(n):
            s, s1 = float(sigmas[i]), float(sigmas[i + 1])
            den = denoise(x, s)
            d = (x - den) / s
            if b == "euler":
                x = x + d * (s1 - s)
            elif b == "euler_a":
                sd, su = self._ancestral(s, s1)
                x = x + d * (sd - s)
                if s1 > 0:
                    x = x + noise() * su
            elif b == "heun":
                if s1 == 0:
                    x = x + d * (s1 - s)
                else:
                    x2 = x + d * (s1 - s)
                    d2 = (x2 - denoise(x2, s1)) / s1
                    x = x + (d + d2) / 2 * (s1 - s)
            elif b in ("dpm_2", "dpm_2_a"):
                sd, su = self._ancestral(s, s1) if b == "dpm_2_a" else (s1, 0.0)
                if sd == 0:
                    x = x + d * (sd - s)
                else:
                    sm = math.exp(0.5 * (math.log(s) + math.log(sd)))
                    x2 = x + d * (sm - s)
                    d2 = (x2 - denoise(x2, sm)) / sm
                    x = x + d2 * (sd - s)
                if su > 0:
                    x = x + noise() * su
            elif b == "lms":
                ds.append(d)
                ds = ds[-4:]
                order = min(i + 1, 4)
                for j in range(order):
                    x = x + _lms_coeff(order, sigmas, i, j) * ds[-1 - j]
            elif b == "dpmpp_2m":
                # DPM-Solver++(2M) in log-sigma time
                if s1 == 0:
                    x = den
                else:
                    t, t1 = -math.log(s), -math.log(s1)
                    h = t1 - t
                    if old_den is None:
                        x = (s1 / s) * x - math.expm1(-h) * den
                    else:
                        r = h_last / h
                        dd = (1 + 1 / (2 * r)) * den - (1 / (2 * r)) * old_den
                        x = (s1 / s) * x - math.expm1(-h) * dd
                    h_last = h
                old_den = den
            elif b == "unipc":
                # UniPC (bh2, data prediction, order 2): the UniC corrector first moves the previous
                # step's point using the model value just computed there, then the UniP predictor
                # steps on (its order-2 form is the DPM-Solver++(2M) update); the final step is first
                # order (the step to sigma 0 returns the data prediction).  Variance-exploding form: the alpha_t factors cancel.
                if pc is not None:
                    xt_, m0, d1, rk, bh, hh = pc
                    d1t = den - m0
                    if d1 is None:
                        x = xt_ - bh * 0.5 * d1t
                    else:
                        r0, r1 = _unic_rhos(rk, hh, bh)
                        x = xt_ - bh * (r0 * d1 + r1 * d1t)
                if s1 == 0:
                    x = den
                    pc = None
                else:
                    t, t1 = -math.log(s), -math.log(s1)
                    h = t1 - t
                    hh = -h
                    bh = math.expm1(hh)
                    xt_ = (s1 / s) * x - math.expm1(hh) * den
                    if old_den is None:
                        d1, rk = None, 0.0
                        x = xt_
                    else:
                        rk = (-math.log(float(sigmas[i - 1])) - t) / h
                        d1 = (old_den - den) / rk
                        x = xt_ - bh * 0.5 * d1
                    pc = (xt_, den, d1, rk, bh, hh)
                old_den = den
            elif b == "dpmpp_sde":
                # DPM-Solver++(2S): a midpoint in log-sigma, deterministic (the singlestep solver
                # the reference's mapping selects)
                if s1 == 0:
                    x = den
                else:
                    t, t1 = -math.log(s), -math.log(s1)
                    h = t1 - t
                    sm = math.exp(-(t + 0.5 * h))
                    x2 = (sm / s) * x - math.expm1(-0.5 * h) * den
                    den2 = denoise(x2, sm)
                    x = (s1 / s) * x - math.expm1(-h) * den2
            elif b == "dpmpp_2m_sde":
                if s1 == 0:
                    x = den
                else:
                    t, t1 = -math.log(s), -math.log(s1)
                    h = t1 - t
                    eta_h = h                                  # eta = 1
                    x = (s1 / s) * math.exp(-eta_h) * x + (-math.expm1(-h - eta_h)) * den
                    if old_den is not None:
                        r = h_last / h
                        x = x + 0.5 * (-math.expm1(-h - eta_h)) * (1 / r) * (den - old_den)
                    x = x + noise() * s1 * math.sqrt(max(-math.expm1(-2 * eta_h), 0.0))
                    h_last = h
                old_den = den
            else:
                raise ValueError(b)
        return x


def _unic_rhos(rk: float, hh: float, bh: float):
    """UniC order-2 weights: solve [[1, 1], [rk, 1]] rho = b with the bh2 phi-function moments."""
    phi = math.expm1(hh) / hh - 1
    b1 = phi / bh
    phi = phi / hh - 0.5
    b2 = phi * 2 / bh
    # rows: rho0 + rho1 = b1 ; rk * rho0 + rho1 = b2
    r0 = (b1 - b2) / (1 - rk)
    return r0, b1 - r0


def _lms_coeff(order: int, sigmas: Sequence[float], i: int, j: int) -> float:
    from scipy import integrate

    def fn(tau):
        prod = 1.0
        for k in range(order):
            if j == k:
                continue
            prod *= (tau - sigmas[i - k]) / (sigmas[i - j] - sigmas[i - k])
        return prod
    return integrate.quad(fn, sigmas[i], sigmas[i + 1], epsrel=1e-4)[0]


class PLMS:
    """PNDM with skip_prk_steps (diffusers PNDMScheduler.step_plms): eps extrapolated from up to
    four previous model outputs, the transfer x_t -> x_prev of the PNDM paper."""

    def __init__(self, c: dict):
        self.ac = train_alphas_cumprod(c)
        self.n_train = len(self.ac)
        self.offset = int(c.get("steps_offset", 1))
        self.final_ac = 1.0 if c.get("set_alpha_to_one", False) else float(self.ac[0])
        self.pred = c.get("prediction_type", "epsilon")

    def timesteps(self, steps: int) -> List[int]:
        r = self.n_train // steps
        ts = [i * r + self.offset for i in range(steps)]
        # diffusers: timesteps[:-1], timesteps[-2:-1], timesteps[-1:] reversed (one extra eval)
        plms = ts[:-1] + ts[-2:-1] + ts[-1:] if steps > 1 else ts
        return plms[::-1]

    def reset(self, steps: int):
        self.ets, self.counter, self.cur = [], 0, None
        self.step_size = self.n_train // steps

    def _prev(self, x, t, tp, eps):
        a = float(self.ac[t])
        ap = float(self.ac[tp]) if tp >= 0 else self.final_ac
        if self.pred == "v_prediction":
            eps = math.sqrt(a) * eps + math.sqrt(1 - a) * x
        coeff = (ap / a) ** 0.5
        denom = a * (1 - ap) ** 0.5 + (a * (1 - a) * ap) ** 0.5
        return coeff * x - (ap - a) * eps / denom

    def step(self, out: torch.Tensor, t: int, x: torch.Tensor) -> torch.Tensor:
        tp = t - self.step_size
        if self.counter != 1:
            self.ets = self.ets[-3:] + [out]
        else:
            tp, t = t, t + self.step_size
        if len(self.ets) == 1 and self.counter == 0:
            e = out
            self.cur = x
        elif len(self.ets) == 1 and self.counter == 1:
            e = (out + self.ets[-1]) / 2
            x, self.cur = self.cur, None
        elif len(self.ets) == 2:
            e = (3 * self.ets[-1] - self.ets[-2]) / 2
        elif len(self.ets) == 3:
            e = (23 * self.ets[-1] - 16 * self.ets[-2] + 5 * self.ets[-3]) / 12
        else:
            e = (55 * self.ets[-1] - 59 * self.ets[-2] + 37 * self.ets[-3] - 9 * self.ets[-4]) / 24
        self.counter += 1
        return self._prev(x, t, tp, e)
