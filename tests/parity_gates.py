"""Shared parity gates for end-to-end (two-pass) renders and training steps.

The reference's sample_pdf is ill-conditioned where the coarse weights put (almost) no mass: its normalised pdf there
is ~1e-5, exactly at the `denom < 1e-5` branch (renderers/utils.py:128-129), and a bin whose pdf is 1e-5..1e-3 turns
an ulp of the CDF into a large move of the sample inside the bin. So an ulp-level difference in the coarse weights can
move a fine sample by up to a bin width, and with it the fine render. The gate therefore splits the rays by their
refined depths:

  * rays whose refined depths (computed from OUR coarse weights) equal the ones computed from the REFERENCE's coarse
    weights (<= z_tol) must match the reference strictly (RGB <= strict, depth <= strict_depth);
  * every other ray must match the reference's fine stage evaluated at OUR refined depths (the oracle's MLP +
    raymarcher on those rays, `fine_at`) just as strictly;
  * and OUR refined depths must be the reference's own refinement (the oracle's RayPointRefiner, renderers/utils.py:
    48-69) applied to OUR coarse weights (<= z_tol, every ray): a flipped ray's depths are then the reference's
    function of coarse weights that the per-stage tests pin to the reference (<= 1e-5), so the loop is closed.

Nothing is gated statistically: every element either matches the reference or is shown to be the reference's own
function of the depths the coarse stage produced. Every gate writes its report (ray counts, flips, maxima) as one JSON
line to gpurun_out/parity_reports.jsonl (merged back from the GPU box; copied to profiles/ per round).
"""
from __future__ import annotations

import json
import os
import time
from pathlib import Path

from contextlib import contextmanager

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
STRICT_GRAD = 1e-4  # north_star's fp32 bound, as max |ours - reference| / max |reference| per gradient tensor
REPORTS = Path(os.environ.get("YANERF_PARITY_REPORTS", ROOT / "gpurun_out" / "parity_reports.jsonl"))



# The bf16 mode stores the weight gradients' X operands H_0..H_7, Y and C as fp8 e4m3 (3 mantissa bits; the reference's
# bf16 autocast keeps them bf16): a weight gradient formed from an fp8 X carries up to e4m3's unit roundoff 2^-4 of
# relative error per term. With few effective points that shows: on mlp_lego's 256 points with random upstream
# gradients the colour-output weights (0.035 vs the autocast's 0.0071), on configs[3]'s full-size step (1024 rays x 64
# coarse points) the coarse layer-5 weights (0.0545 vs 0.0222); at configs[1]'s 786k fine points 0.0018 / 0.0043 vs
# 0.0027 / 0.0043. So in the bf16 (fp8-storage) mode these tensors' bound is at least FP8_UNIT; the all-bf16 mode
# (bf16s) keeps the autocast-derived bound alone.
FP8_UNIT = 2.0 ** -4
FP8_X_WEIGHTS = tuple(f"xyz_encoder.mlp.{i}.0.weight" for i in range(1, 8)) + (
    "intermediate_linear.weight", "color_layer.0.weight", "color_layer.2.weight")


def write_report(kind: str, tag: str, report: dict) -> None:
    """Append one JSON line {kind, tag, time, **report} to the parity report file."""
    try:
        REPORTS.parent.mkdir(parents=True, exist_ok=True)
        with open(REPORTS, "a") as f:
            f.write(json.dumps(dict(kind=kind, tag=tag, time=time.strftime("%Y-%m-%dT%H:%M:%S"), **report)) + "\n")
    except OSError:  # a read-only checkout: the assertion is what gates
        pass


def oracle_fine_at(O, params_f, arch, origins, directions, raymarch_opts, bg=(0.0, 0.0, 0.0)):
    """fine_at(rows, z) -> (rgb [n,3], depth [n]): the oracle's fine MLP + raymarcher on rays `rows` at depths z."""
    origins = np.asarray(origins, np.float32).reshape(-1, 3)
    directions = np.asarray(directions, np.float32).reshape(-1, 3)

    def fine_at(rows, z):
        o, d = origins[rows], directions[rows]
        s, c, _ = O.nerf_mlp_forward(params_f, arch, o, d, z)
        f, dep, _, _, _ = O.raymarch_forward(s, c, z, d, raymarch_opts, default_bg=bg)
        return f, np.asarray(dep).reshape(-1)

    return fine_at


def sensitivity_trials(sens, z_tol=2e-5):
    """Per trial family of make_golden.gen_sensitivity, the rays whose refined depths the REFERENCE itself moves by
    more than z_tol under that equally valid fp32 evaluation of its coarse stage (boolean masks over the rays):
    f64 = float64 end to end; ulp_reorder = exp one ulp off, coarse parameters one ulp off, Linear K-sums split;
    hip_arithmetic = the coarse stage in the fp32 HIP kernels' own arithmetic (MFMA chain of every Linear, correctly
    rounded embedding and capping exp, the composite's operation order; and the MFMA order alone); weights = the
    coarse weights moved by the measured |this build - reference| magnitude (sens["weight_delta"])."""
    out = {"f64": np.abs(np.asarray(sens["z_fine_f64"], np.float64) - sens["z_fine"]).max(-1) > z_tol,
           "ulp_reorder": np.asarray(sens["max_z_move"]) > z_tol}
    if "max_z_move_hip_order" in sens:
        out["hip_arithmetic"] = np.asarray(sens["max_z_move_hip_order"]) > z_tol
    if "max_z_move_weights" in sens:
        out["weights"] = np.asarray(sens["max_z_move_weights"]) > z_tol
    return out


def reference_sensitive_rays(sens, z_tol=2e-5):
    """The union of sensitivity_trials: every ray the reference itself moves under some equally valid fp32
    evaluation of its coarse stage."""
    m = None
    for v in sensitivity_trials(sens, z_tol).values():
        m = v if m is None else (m | v)
    return m


def split_gate(rgb, rgb_ref, z, z_ref, depth=None, depth_ref=None, *, fine_at=None, coarse=None, strict=1e-5,
               strict_depth=1e-4, z_tol=2e-5, tag="", sensitivity=None, same_tol=None, same_tol_depth=None,
               all_vs_oracle=False, hip_exact=False, max_outside_without_weights=0):
    """coarse = (O, lengths [R,Pc], our coarse weights [R,Pc], n_fine): the oracle refinement of our coarse weights
    (deterministic, as the evaluation pass runs it) must equal z on every ray.
    same_tol / same_tol_depth: the bound on the rays whose refined depths agree with the reference's to z_tol (default
    strict / strict_depth). all_vs_oracle: every ray (not only those with other depths) is also held to strict /
    strict_depth against the oracle's fine stage at OUR refined depths -- for a sharp trained density, where depths
    equal to z_tol still move the colour by more than `strict` (the looser same_tol then bounds that effect).
    sensitivity = the reference's own sensitivity golden of this render (reference_sensitive_rays): every ray whose
    refined depths differ between this build and the reference must lie in the set the reference itself moves under
    equally valid fp32 evaluations of its coarse stage (set membership, asserted: none outside).
    hip_exact (the fp32 mode, whose coarse weights the golden's hip-arithmetic trial reproduces bit for bit): the rays
    with other depths must lie in that one trial's set -- the reference's own refinement of this build's coarse weights
    moves exactly them.
    max_outside_without_weights: how many of those rays may lie outside every trial EXCEPT the weight-perturbation one
    (trial (f) perturbs by this build's own measured coarse-weight error, so it is a diagnostic, not a bound on that
    error): 0 in every mode but fp32x3 at the trained weights, whose bf16 MFMA is no IEEE fp32 sequence (measured 2 of
    625 rays, round 5; the bound is that measurement, so a regression fails)."""
    R = len(z)
    rgb = np.asarray(rgb, np.float64).reshape(R, -1)
    rgb_ref = np.asarray(rgb_ref, np.float64).reshape(R, -1)
    z, z_ref = np.asarray(z, np.float32).reshape(R, -1), np.asarray(z_ref, np.float32).reshape(R, -1)
    zerr = np.abs(z.astype(np.float64) - z_ref).max(axis=-1)
    same = zerr <= z_tol
    flip = np.nonzero(~same)[0]
    err = np.abs(rgb - rgb_ref).max(axis=-1)
    report = dict(rays=R, rays_with_other_depths=int(flip.size), rgb_above_1e4=int((err > 1e-4).sum()),
                  max_rgb_err_same_depths=float(err[same].max()) if same.any() else 0.0,
                  max_rgb_err_other_depths_vs_reference=float(err[flip].max()) if flip.size else 0.0)
    if depth is not None:
        depth = np.asarray(depth, np.float64).reshape(-1)
        derr = np.abs(depth - np.asarray(depth_ref, np.float64).reshape(-1))
        report["max_depth_err_same_depths"] = float(derr[same].max()) if same.any() else 0.0
    if sensitivity is not None:
        sens = reference_sensitive_rays(sensitivity, z_tol)
        assert sens.shape == same.shape, (sens.shape, same.shape)
        trials = sensitivity_trials(sensitivity, z_tol)
        report.update(reference_sensitive_rays=int(sens.sum()),
                      reference_moved_by_f64=int(trials["f64"].sum()),
                      reference_moved_by_trial={k: int(v.sum()) for k, v in trials.items()},
                      other_depths_within_trial={k: int((~same & v).sum()) for k, v in trials.items()},
                      rays_with_other_depths_outside_reference_sensitive=int((~same & ~sens).sum()),
                      outside_without_weights_trial=int((~same & ~(trials["f64"] | trials["ulp_reorder"] | trials.get(
                          "hip_arithmetic", np.zeros_like(same)))).sum()))
        if hip_exact:
            report["outside_hip_arithmetic_trial"] = int((~same & ~trials["hip_arithmetic"]).sum())
    if coarse is not None:
        O, zc, w_ours, n_fine = coarse
        zc = np.asarray(zc, np.float32).reshape(R, -1)
        z_or = O.refine(zc, np.asarray(w_ours, np.float32).reshape(R, -1), int(n_fine), random_sampling=False)
        report["max_depth_err_vs_oracle_refine_of_our_weights"] = float(np.abs(z.astype(np.float64) - z_or).max())
    if flip.size and fine_at is not None:
        f_o, d_o = fine_at(flip, z[flip])
        e2 = np.abs(rgb[flip] - np.asarray(f_o, np.float64).reshape(flip.size, -1)).max(axis=-1)
        report["max_rgb_err_other_depths_vs_oracle_at_our_depths"] = float(e2.max())
        if depth is not None:
            report["max_depth_err_other_depths_vs_oracle_at_our_depths"] = float(
                np.abs(depth[flip] - np.asarray(d_o, np.float64)).max())
    if all_vs_oracle:
        rows = np.arange(R)
        f_a, d_a = fine_at(rows, z)
        report["max_rgb_err_all_vs_oracle_at_our_depths"] = float(
            np.abs(rgb - np.asarray(f_a, np.float64).reshape(R, -1)).max())
        if depth is not None:
            report["max_depth_err_all_vs_oracle_at_our_depths"] = float(np.abs(depth - np.asarray(d_a, np.float64)).max())
    report["other_depth_rays"] = [int(i) for i in flip]
    if sensitivity is not None:
        report["outside_reference_sensitive_rays"] = [int(i) for i in np.nonzero(~same & ~sens)[0]]
    dump = os.environ.get("YANERF_PARITY_DUMP")
    if dump:  # the inputs of this gate, for offline analysis of the flipped rays (tools/, not a gate)
        Path(dump).mkdir(parents=True, exist_ok=True)
        np.savez(Path(dump) / (tag.replace(" ", "_") + ".npz"), z=z, z_ref=z_ref, rgb=rgb, rgb_ref=rgb_ref,
                 w_coarse=np.asarray(coarse[2], np.float32) if coarse is not None else np.zeros(0, np.float32))
    print(f"split_gate {tag}: {report}")
    write_report("split_gate", tag, report)
    assert report["max_rgb_err_same_depths"] <= (strict if same_tol is None else same_tol), report
    if depth is not None:
        assert report["max_depth_err_same_depths"] <= (strict_depth if same_tol_depth is None else same_tol_depth), report
    if all_vs_oracle:
        assert report["max_rgb_err_all_vs_oracle_at_our_depths"] <= strict, report
        if depth is not None:
            assert report["max_depth_err_all_vs_oracle_at_our_depths"] <= strict_depth, report
    if coarse is not None:
        assert report["max_depth_err_vs_oracle_refine_of_our_weights"] <= z_tol, report
    if sensitivity is not None:
        # set membership: the reference itself moves every one of these rays under some valid fp32 evaluation
        assert report["rays_with_other_depths_outside_reference_sensitive"] == 0, report
        assert report["outside_without_weights_trial"] <= max_outside_without_weights, report
        if hip_exact:
            assert report["outside_hip_arithmetic_trial"] == 0, report
    if flip.size:
        assert fine_at is not None, f"{flip.size} rays with other refined depths and no fine_at to account for them"
        assert coarse is not None, f"{flip.size} rays with other refined depths: pass `coarse` to close the loop"
        assert report["max_rgb_err_other_depths_vs_oracle_at_our_depths"] <= strict, report
        if depth is not None:
            assert report["max_depth_err_other_depths_vs_oracle_at_our_depths"] <= strict_depth, report
    return report


# fp32 summation order. Every parameter-gradient element is a sum over the step's points (up to ~25k terms here), and
# two correct fp32 evaluations summing the same terms in different orders differ by up to ~n * 2^-24 * sum|terms|.
# Where a sum cancels (sum|terms| >> |sum|: the density-layer bias at the trained weights, kappa ~15) that difference
# alone can exceed 1e-4 * max|ref| with both sides correct -- there the reference's own value sits 7.8e-6 * sum|terms|
# from the exact (float64) sum of its terms, 1.1e-4 of its magnitude. Every strict gradient gate therefore allows, per
# element, SUM_REL * sum|terms| on top of its relative bound (sum|terms| from the oracle, nerf_mlp_backward abs_terms),
# and reports how many elements needed it ("sum_limited").
SUM_REL = 2e-5


def _flat(x, idx=None):
    x = np.asarray(x, np.float64).reshape(-1)
    return x if idx is None else x[idx]


# an fp32 implementation's gradients may be at most this much further from the exact (float64) algorithm than the
# reference's own fp32 gradients are (or within STRICT_GRAD of it)
EXACT_RATIO = 1.5


@contextmanager
def float64_oracle(O):
    """Run the oracle in float64 (its arithmetic type is the module global `f32`): the reference's algorithm without
    fp32 rounding, the common yardstick for how far each fp32 implementation (the reference, the oracle, HIP) lands
    from the exact result."""
    old = O.f32
    O.f32 = np.float64
    try:
        yield O
    finally:
        O.f32 = old


def max_rel_vs(models_or_items, exact) -> float:
    """max over tensors of max |x - exact| / max |exact| (exact: {name: array}); items are (name, array) pairs."""
    worst = 0.0
    for name, x in models_or_items:
        e = np.asarray(exact[name], np.float64).reshape(-1)
        x = np.asarray(x, np.float64).reshape(-1)
        worst = max(worst, float(np.abs(x - e).max() / max(np.abs(e).max(), 1e-30)))
    return worst


def strict_grad_gate(v, ref, abs_terms=None, name="", tol: float = STRICT_GRAD) -> dict:
    """|v - ref| <= tol * max|ref| + SUM_REL * sum|terms| for every element (abs_terms None: the relative bound alone).
    Returns {err: max |v - ref| / max|ref|, sum_limited: elements beyond tol * max|ref|}."""
    v, ref = _flat(v), _flat(ref)
    M = max(np.abs(ref).max(), 1e-30)
    err = np.abs(v - ref)
    allow = tol * M + (SUM_REL * _flat(abs_terms) if abs_terms is not None else 0.0)
    over = err > tol * M
    # the share of the summation allowance used by the worst element beyond the relative bound (0..1)
    rep = dict(err=float(err.max() / M), sum_limited=int(over.sum()),
               sum_allowance_used=float(((err - tol * M)[over] / np.maximum(SUM_REL * _flat(abs_terms)[over], 1e-300))
                                        .max()) if abs_terms is not None and over.any() else 0.0)
    assert (err <= allow).all(), (name, rep)
    return rep


def grad_err(v, ref) -> float:
    """max |v - ref| / max |ref| (elementwise, relative to the tensor's largest gradient)."""
    v, ref = np.asarray(v, np.float64), np.asarray(ref, np.float64)
    return float(np.abs(v - ref).max() / max(np.abs(ref).max(), 1e-30))


def loose_grad_gate(v, ref, name, enforce: bool = True):
    """The end-to-end statistical view of gradients that sum over rays whose refined depths may have flipped
    (split_gate): >= 98 % of elements within 5e-3 * max, all within 3e-2 * max. Returns the relative L2 error. The
    parity tests report it (enforce=False) beside the strict per-element tie-budget gate below."""
    v, ref = np.asarray(v, np.float64), np.asarray(ref, np.float64)
    mx = np.abs(ref).max()
    err = np.abs(v - ref)
    if enforce:
        assert err.max() <= 3e-2 * mx, (name, err.max() / mx)
        assert (err <= 5e-3 * mx).mean() >= 0.98, (name, (err <= 5e-3 * mx).mean())
    return float(np.linalg.norm(v - ref) / max(np.linalg.norm(ref), 1e-30))


# the oracle's gradients under the reference's own ReLU decisions and refined depths against the reference's
# (test_oracle_golden.test_train_step_lego_strict_under_reference_relu_decisions: measured 7.5e-6 coarse, 1.6e-5 fine)
ORACLE_PIN = 2e-5


def golden_grad_items(g, models):
    """(model index, name, ours, reference, index into the flattened tensor or None) for every parameter gradient the
    train-step golden holds: whole tensors up to 4,096 elements, a fixed sample of 256 entries of the larger ones."""
    for i, m in enumerate(models):
        for name, p in m.named_parameters():
            v = p.grad.detach().float().cpu().numpy().astype(np.float64).reshape(-1)
            if f"grad{i}:{name}" in g:
                yield i, name, v, g[f"grad{i}:{name}"].astype(np.float64).reshape(-1), None
            else:
                idx = g[f"gradidx{i}:{name}"]
                yield i, name, v[idx], g[f"gradval{i}:{name}"].astype(np.float64), idx


def tie_budget_gate(v, ref, o_hip, o_ref, name, strict: float = STRICT_GRAD, pin: float = ORACLE_PIN,
                    abs_terms=None) -> dict:
    """The direct comparison with the reference's gradient, strict per element with the ReLU ties (and, for a fine pass
    at this build's own refined depths, the sample_pdf flips) as an explicit budget:

        |ours - reference| <= strict * max|reference| + |O_hip - O_ref|     (every element)

    O_hip = the reference's algorithm (oracle) under the ReLU decisions this build took (at its refined depths),
    O_ref = the same under the reference's own recorded decisions (at the reference's depths), itself pinned to the
    reference (|O_ref - reference| <= pin * max, asserted here). |O_hip - O_ref| is exactly what the differing decisions
    (fp32 ties at the kink, flipped samples) contribute; whatever ours differs by beyond it must be within `strict`.
    Both bounds also allow SUM_REL * sum|terms| per element (abs_terms: the oracle's, under the reference's decisions),
    the fp32 summation-order term (see SUM_REL). Returns {direct, budget, residual, pin, sum_limited}: max |ours - ref|,
    max |O_hip - O_ref|, max (|ours - ref| - |O_hip - O_ref|) and max |O_ref - ref|, each relative to max |ref|, and
    the number of elements beyond the relative bounds alone."""
    v, ref, o_hip, o_ref = (np.asarray(x, np.float64).reshape(-1) for x in (v, ref, o_hip, o_ref))
    M = max(np.abs(ref).max(), 1e-30)
    slack = SUM_REL * _flat(abs_terms) if abs_terms is not None else 0.0
    pin_abs = np.abs(o_ref - ref)
    pin_err = float(pin_abs.max() / M)
    assert (pin_abs <= pin * M + slack).all(), (name, "oracle under the reference's decisions vs the reference", pin_err)
    budget = np.abs(o_hip - o_ref)
    direct = np.abs(v - ref)
    excess = direct - budget
    over = excess > strict * M
    rep = dict(direct=float(direct.max() / M), budget=float(budget.max() / M),
               residual=float(max(excess.max(), 0.0) / M), pin=pin_err,
               sum_limited=int(over.sum()), pin_sum_limited=int((pin_abs > pin * M).sum()))
    assert (excess <= strict * M + slack).all(), (name, rep)
    return rep


def summarize_tie_budget(per_tensor: dict) -> dict:
    """Per model: the worst direct error, tie budget and residual over its tensors (for the parity report)."""
    out = {}
    for i in sorted({k[0] for k in per_tensor}):
        rows = [r for k, r in per_tensor.items() if k[0] == i]
        tag = "coarse" if i == 0 else "fine"
        out[f"{tag}_direct_max"] = max(r["direct"] for r in rows)
        out[f"{tag}_tie_budget_max"] = max(r["budget"] for r in rows)
        out[f"{tag}_residual_max"] = max(r["residual"] for r in rows)
        out[f"{tag}_oracle_pin_max"] = max(r["pin"] for r in rows)
        out[f"{tag}_sum_limited_elements"] = sum(r.get("sum_limited", 0) for r in rows)
        out[f"{tag}_pin_sum_limited_elements"] = sum(r.get("pin_sum_limited", 0) for r in rows)
    out["per_tensor"] = {f"{k[0]}:{k[1]}": {kk: float(f"{vv:.3e}") for kk, vv in r.items()}
                         for k, r in per_tensor.items()}
    return out


def golden_grad_pairs(g, models):
    """(model index, name, ours, reference) for every parameter gradient the train-step golden holds: whole tensors up
    to 4,096 elements, a fixed sample of 256 entries (plus the norm) of the larger ones."""
    for i, m in enumerate(models):
        for name, p in m.named_parameters():
            v = p.grad.detach().float().cpu().numpy().astype(np.float64)
            if f"grad{i}:{name}" in g:
                yield i, name, v, g[f"grad{i}:{name}"].astype(np.float64), None
            else:
                idx = g[f"gradidx{i}:{name}"]
                yield i, name, v.reshape(-1)[idx], g[f"gradval{i}:{name}"].astype(np.float64), (
                    np.linalg.norm(v), float(g[f"gradsum{i}:{name}"][1]))


# ------------------------------------------------------------------------------------------- ReLU ties
TIE_REL = 5e-5  # a ReLU decision may differ only where |pre-activation| <= TIE_REL * max |pre-activation| of its layer


def hip_relu_masks(saved, n_points: int, n_layers: int = 8, hidden: int = 256, hidden_dir: int = 128):
    """The ReLU decisions the HIP forward took, read back from its saved activations (fp32 and fp32x3 modes: feature-
    major fp32 rows, post-ReLU values, so decision = value > 0). Test-side mirror of csrc/mlp.hip `saved_rows` /
    `row_ld` / `npad_of` (64-point tiles; rows PE 64 | H_0..H_{L-1} 256 each | Y 256 | dirPE 32 | C 128, each row an
    odd multiple of 256 bytes long). A wrong mirror shows up as thousands of disagreements with the oracle's signs."""
    import torch
    npad = -(-n_points // 64) * 64
    units = (npad * 4 + 255) // 256
    if units % 2 == 0:
        units += 1
    ld = units * 256 // 4
    rows = 64 + 256 * n_layers + 256 + 32 + 128
    f = saved[: rows * ld * 4].view(torch.float32).view(rows, ld)[:, :n_points].cpu().numpy()
    trunk = [f[64 + 256 * li: 64 + 256 * li + hidden].T > 0 for li in range(n_layers)]
    c0 = 64 + 256 * n_layers + 256 + 32
    return dict(trunk=trunk, color=f[c0: c0 + hidden_dir].T > 0)


def golden_relu_masks(g, k: int):
    """The reference's ReLU decisions of pass k recorded in train_step_lego.npz (make_golden.gen_train_step)."""
    return dict(trunk=[np.unpackbits(g[f"relu{k}:trunk"][li], axis=-1).astype(bool)
                       for li in range(g[f"relu{k}:trunk"].shape[0])],
                color=np.unpackbits(g[f"relu{k}:color"], axis=-1).astype(bool))


def relu_ties(masks, other, cache):
    """Units where two sets of ReLU decisions of the same network on the same points disagree, and the largest
    |pre-activation| among them relative to its layer's largest (from the oracle's forward `cache`). Every
    disagreement must be an fp32 tie at the kink (<= TIE_REL): two correct fp32 evaluations with different summation
    orders can put a pre-activation within rounding of zero on either side. Returns (count, worst relative |z|)."""
    n, worst = 0, 0.0
    pairs = list(zip(masks["trunk"], other["trunk"], cache.layer_pre)) + [(masks["color"], other["color"],
                                                                            cache.c0_pre)]
    for a, b, z in pairs:
        d = np.asarray(a, bool) != np.asarray(b, bool).reshape(np.shape(a))
        if d.any():
            za = np.abs(np.asarray(z)).reshape(d.shape)
            n += int(d.sum())
            worst = max(worst, float(za[d].max() / max(za.max(), 1e-30)))
    return n, worst
