"""Full-length token agreement at the benchmarked shape: the 32-slot engine runs
bench.py's 32 config-3 requests (DIMS_04B bf16, 32 global + 512 fixed semantic tokens) and two
zero-shot requests on the fp16 model with the reference RAF fixtures' global tokens; their
token streams are compared with the oracle's (tests/golden/fulllength_tokens.json, made by
tests/golden/make_fulllength_golden.py).

The GPU and the oracle agree on logits to ~1e-4 (different f32 summation orders), so identical
tokens over hundreds of sampled steps are a measured outcome, not a guarantee. Where a stream
diverges, the test finds the first divergent step, teacher-forces the oracle's tokens through
the GPU (RnnOption::Full, bitwise the logits the decode saw: batch- and chunk-invariant) and
checks that (a) every logit before and at that step is within LOGIT_ATOL of the oracle's and
(b) the exact sampler applied to the GPU's logits at that step, with the request's own draw,
gives the GPU's token -- i.e. the divergence is the fp difference in the logits flipping a
near-tie, not a sampler or controller difference. First-divergence steps and logit gaps are
written to $RWKVTTS_REPORT_DIR/fulllength_report.json when that variable is set.

Gates: the prefix logit gap stays under LOGIT_ATOL = 2e-4 (about 4x the 5.3e-5
measured at round 3, profiles/r03a_fulllength_report.json), no stream diverges before its
MIN_DIV_STEP-th sampled token (global + semantic steps), and at least MIN_EXACT of the 8 streams
(6 normal-mode, 2 zero-shot) are token-exact over their whole length."""
import json
import os

import numpy as np
import pytest

import rwkvtts
from rwkvtts import weights as W
from helpers import to_struct

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "fulllength_tokens.json")
LOGIT_ATOL = 2e-4
MIN_DIV_STEP = 300
MIN_EXACT = 7
_REPORTS = {}  # test name -> its reports (the summary test counts exact streams over both)


def _bench_requests():
    """bench.py requests(step=0) at rank 0 (rid = i)."""
    reqs = []
    for i in range(32):
        rs = np.random.RandomState(i)
        text = rs.randint(12293, 77822, size=24).tolist()
        reqs.append(rwkvtts.TtsBatchRequest(text_tokens=text, property_tokens=[77823, 77838, 77869, 77845, 77830, 77826],
                                            args=rwkvtts.SamplerArgs(seed=i, max_tokens=2048), fixed_semantic=512))
    return reqs


def _req_from(e, raf=None):
    return rwkvtts.TtsBatchRequest(text_tokens=e["text"], property_tokens=e["props"],
                                   ref_global_tokens=None if raf is None else raf["global_tokens"],
                                   ref_semantic_tokens=None if raf is None else raf["semantic_tokens"],
                                   args=rwkvtts.SamplerArgs(seed=e["seed"], max_tokens=2048),
                                   fixed_semantic=e["fixed_semantic"])


def _first_div(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i
    return None if len(a) == len(b) else min(len(a), len(b))


def _explain(blob, rt, req, e, got, zero_shot):
    """First divergence of (global, semantic) vs the fixture, with the teacher-forced logit gap."""
    import oracle
    g_ref, s_ref = e["global"], e["semantic"]
    dg = None if zero_shot else _first_div(got[0], g_ref)
    ds = _first_div(got[1], s_ref)
    if dg is None and ds is None:
        return {"name": e["name"], "exact": True, "steps": len(g_ref) + len(s_ref)}
    # the token sequence fed after the prompt, up to and including the divergent step's input
    q, keep = to_struct(req)
    prompt = list(req.property_tokens) + [rwkvtts.TAG_2] + list(req.text_tokens) + [rwkvtts.TAG_0]
    if zero_shot:
        prompt += [min(max(x, 0), 4095) + 8196 for x in req.ref_global_tokens] + [rwkvtts.TAG_1]
    if dg is not None:
        fed = [x + 8196 for x in g_ref[:dg]]
        step, head, phase = dg, 4096, "global"
    else:
        fed = ([] if zero_shot else [x + 8196 for x in g_ref] + [rwkvtts.TAG_1]) + list(s_ref[:ds])
        step, head, phase = ds, 8193, "semantic"
    seq = prompt + fed
    rt.reset_slot(0)
    inp = rwkvtts.RnnInput([rwkvtts.RnnInputBatch(list(seq), rwkvtts.RnnOption.Full)], 4096)
    _, out = rt.infer(inp, head_rows=8193, slots=[0])
    gpu = out[0].reshape(len(seq), -1)
    om = oracle.Model(blob)
    st = om.new_state()
    gaps = []
    first_lg = len(prompt) - 1
    for t, tok in enumerate(seq):
        ref = om.forward(st, tok, 8193 if t >= first_lg else 0)
        if t >= first_lg:
            gaps.append(float(np.abs(gpu[t] - ref).max()))
            last_ref = ref
    gl = gpu[-1][:head].copy()
    orl = last_ref[:head].copy()
    if phase == "semantic" and req.fixed_semantic > 0:  # fixed-length mode masks EOS (controller.c)
        gl[8192] = orl[8192] = -np.inf
    # the request's draw at this step: global stream seed+1000 draw dg, semantic stream seed+2000
    # draw ds (zero-shot: seed+2000, one draw per step unless a window re-draw happened before)
    seed = req.args.seed + (1000 if phase == "global" else 2000)
    rng = oracle.Rng(seed)
    for _ in range(step):
        rng.gen_f32()
    k = 20 if phase == "global" else 80
    samp_gpu = oracle.sample(gl, 1.0, 0.95, k, None, rng)
    return {"name": e["name"], "exact": False, "phase": phase, "first_divergence_step": step,
            "steps_compared": len(g_ref) + len(s_ref), "gpu_token": (got[0] if phase == "global" else got[1])[step],
            "oracle_token": (g_ref if phase == "global" else s_ref)[step],
            "oracle_sampler_on_gpu_logits": int(samp_gpu), "max_logit_gap_prefix": max(gaps),
            "logit_gap_at_divergence": gaps[-1],
            "logit_gap_at_divergence_head": _finite_gap(gl, orl)}


def _finite_gap(a, b):
    """max |a - b| over the entries finite in both (masked -inf entries compared first, so no
    -inf - -inf = nan is ever formed)"""
    m = np.isfinite(a) & np.isfinite(b)
    return float(np.abs(a[m] - b[m]).max()) if m.any() else 0.0


def _check(reports, key):
    _REPORTS[key] = reports
    d = os.environ.get("RWKVTTS_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, "fulllength_report.json")
        old = json.load(open(path)) if os.path.exists(path) else []
        json.dump(old + reports, open(path, "w"), indent=1)
    for r in reports:
        if r["exact"]:
            continue
        assert r["max_logit_gap_prefix"] < LOGIT_ATOL, r
        # the step index over the whole stream: normal-mode semantic steps follow 32 global ones
        total = r["first_divergence_step"] + (32 if (r["phase"] == "semantic" and not r["name"].startswith("zero_shot")) else 0)
        assert total >= MIN_DIV_STEP, ("divergence too early", r)
        # zero-shot window re-draws shift the draw index: the sampler check applies to normal mode
        if not r["name"].startswith("zero_shot"):
            assert r["oracle_sampler_on_gpu_logits"] == r["gpu_token"], r


@pytest.fixture(scope="module")
def gold():
    return json.load(open(GOLDEN))


def test_bench_requests_full_length(gold):
    blob = W.synth_blob(W.DIMS_04B, seed=20251205)
    rt = rwkvtts.SharedRwkvRuntime(blob, max_slots=32, token_chunk_size=2048, use_graphs=True)
    try:
        reqs = _bench_requests()
        got = rt.generate_batch(reqs)
        reports = []
        for e in gold["normal"]["requests"]:
            rid = int(e["name"].split("rid")[1])
            assert reqs[rid].text_tokens == e["text"] and reqs[rid].args.seed == e["seed"]
            reports.append(_explain(blob, rt, reqs[rid], e, got[rid], False))
    finally:
        rt.close()
    _check(reports, "normal")


def test_zero_shot_full_length(gold):
    blob = W.synth_blob(W.DIMS_04B, seed=20251205, dtype=rwkvtts._ffi.DTYPE_F16)
    rt = rwkvtts.SharedRwkvRuntime(blob, max_slots=32, token_chunk_size=2048, use_graphs=True)
    gdir = os.path.dirname(GOLDEN)
    try:
        es = gold["zero_shot"]["requests"]
        reqs = [_req_from(e, json.load(open(os.path.join(gdir, e["raf"])))) for e in es]
        got = rt.generate_batch(reqs)
        reports = [_explain(blob, rt, r, e, gs, True) for r, e, gs in zip(reqs, es, got)]
        for (g, _), e in zip(got, es):
            assert g == e["global"]  # the reference's own 32 global tokens come back
    finally:
        rt.close()
    _check(reports, "zero_shot")


def test_full_length_exact_stream_count():
    """At least MIN_EXACT of the 8 streams token-exact (runs after the two tests above)."""
    if set(_REPORTS) != {"normal", "zero_shot"}:
        pytest.skip("needs both full-length tests in this session")
    reps = _REPORTS["normal"] + _REPORTS["zero_shot"]
    assert len(reps) == 8
    exact = sum(1 for r in reps if r["exact"])
    assert exact >= MIN_EXACT, [r for r in reps if not r["exact"]]
