"""Pointwise parity of the gfx950 physics (analytic gradients) against the oracle's
dual-number restatement: func!/func_axion! (RayTracer.jl:71-123), hamiltonian
(:530-556) and the resonance condition (:254-298). FP64, relative tolerance 1e-10 on
each component against the component scale."""
import numpy as np
import pytest

from conftest import CONFIGS, random_states

pytestmark = pytest.mark.gpu

N = 2048


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available()
    return torch


def _engine(kw):
    from adiabatic_raytracer_amd import Engine, Params
    return Engine(Params(**kw))


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
@pytest.mark.parametrize("species", [1, 0])
def test_rhs_matches_oracle(cfg, species, torch_mod, oracle_lib):
    torch = torch_mod
    kw = CONFIGS[cfg]
    eng = _engine(kw)
    p = oracle_lib.make_params(**kw)
    U, tau = random_states(N, seed=1 + species)
    erg = np.full(N, 1.0000002692622573e-05)
    dev = lambda a, dt=torch.float64: torch.tensor(np.ascontiguousarray(a), dtype=dt, device="cuda")  # noqa: E731
    du = eng.eval_rhs(dev(U.reshape(-1)), dev(tau), dev(erg), dev(np.full(N, species), torch.int8))
    du = du.cpu().numpy().reshape(7, N)
    ref = np.stack([oracle_lib.rhs(p, species, U[:, i], tau[i], erg[i]) for i in range(N)], axis=1)
    scale = np.abs(ref).max(axis=1, keepdims=True) + 1e-300
    err = np.abs(du - ref) / scale
    assert np.nanmax(err) < 1e-10, (cfg, species, np.nanmax(err, axis=1))


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_condition_matches_oracle(cfg, torch_mod, oracle_lib):
    torch = torch_mod
    kw = CONFIGS[cfg]
    eng = _engine(kw)
    p = oracle_lib.make_params(**kw)
    U, tau = random_states(N, seed=7)
    dev = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda")  # noqa: E731
    c = eng.eval_condition(dev(U.reshape(-1)), dev(tau)).cpu().numpy()
    ref = np.array([oracle_lib.condition(p, U[:, i], tau[i]) for i in range(N)])
    both = ~np.isnan(ref)
    assert np.array_equal(np.isnan(c), np.isnan(ref))
    err = np.abs(c[both] - ref[both]) / (np.abs(ref[both]) + 1e-12)
    j = np.flatnonzero(both)[np.argmax(err)]
    assert err.max() < 1e-9, (err.max(), int(j), c[j], ref[j], U[:, j].tolist(), tau[j])


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_hamiltonian_matches_oracle(cfg, torch_mod, oracle_lib):
    torch = torch_mod
    kw = CONFIGS[cfg]
    eng = _engine(kw)
    p = oracle_lib.make_params(**kw)
    U, tau = random_states(N, seed=11, rmin=9.0)  # includes r < rNS (the clamp, RayTracer.jl:531)
    erg = 1.0000002692622573e-05
    x, k = U[0:3], U[3:6] * erg
    T = np.exp(tau)
    E = -U[6]
    dev = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda")  # noqa: E731
    H, gx, gk, gT = [a.cpu().numpy() for a in eng.eval_hamiltonian(dev(x.reshape(-1)), dev(k.reshape(-1)), dev(T),
                                                                    dev(E))]
    gx, gk = gx.reshape(3, N), gk.reshape(3, N)
    for i in range(N):
        h, rx, rk, rT = oracle_lib.hamiltonian(p, x[:, i], k[:, i], T[i], E[i])
        s = abs(h) + 1e-30
        assert abs(H[i] - h) <= 1e-9 * max(s, E[i] ** 2), (i, H[i], h)
        for a, b in ((gx[:, i], rx), (gk[:, i], rk)):
            assert np.all(np.abs(a - b) <= 1e-9 * (np.abs(b).max() + 1e-300)), (cfg, i, a, b)
        assert abs(gT[i] - rT) <= 1e-9 * (abs(rT) + np.abs(rx).max() * 1e-3 + 1e-300), (cfg, i, gT[i], rT)


# The non-default physics branches on the device: the boundary layer of plasma
# (RayTracer.jl:1155-1162; func! applies it to the ∂t pass only, :84-88) and isotropic
# plasma (k∥ -> 0, :542-543 and the condition's :1573-1575 analogue).
BRANCHES = {"bndry_lyr": dict(bndry_lyr=3.0), "isotropic": dict(isotropic=True)}


@pytest.mark.parametrize("cfg", ["flat", "gr"])
@pytest.mark.parametrize("branch", sorted(BRANCHES))
def test_branch_rhs_and_condition_match_oracle(cfg, branch, torch_mod, oracle_lib):
    torch = torch_mod
    kw = dict(CONFIGS[cfg], **BRANCHES[branch])
    eng = _engine(kw)
    p = oracle_lib.make_params(**kw)
    U, tau = random_states(N, seed=21, rmin=9.5)
    erg = np.full(N, 1.0000002692622573e-05)
    dev = lambda a, dt=torch.float64: torch.tensor(np.ascontiguousarray(a), dtype=dt, device="cuda")  # noqa: E731
    du = eng.eval_rhs(dev(U.reshape(-1)), dev(tau), dev(erg), dev(np.full(N, 1), torch.int8)).cpu().numpy()
    du = du.reshape(7, N)
    ref = np.stack([oracle_lib.rhs(p, 1, U[:, i], tau[i], erg[i]) for i in range(N)], axis=1)
    scale = np.abs(ref).max(axis=1, keepdims=True) + 1e-300
    assert np.nanmax(np.abs(du - ref) / scale) < 1e-10, (cfg, branch, np.nanmax(np.abs(du - ref) / scale, axis=1))
    c = eng.eval_condition(dev(U.reshape(-1)), dev(tau)).cpu().numpy()
    cr = np.array([oracle_lib.condition(p, U[:, i], tau[i]) for i in range(N)])
    assert np.array_equal(np.isnan(c), np.isnan(cr))
    ok = ~np.isnan(cr)
    assert np.max(np.abs(c[ok] - cr[ok]) / (np.abs(cr[ok]) + 1e-3)) < 1e-9
