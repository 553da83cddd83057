"""Kernel routing of a training step — the ONE table of which kernel runs which op.

Every shape-dependent kernel choice of the framework reads its setting here (``get``), so what a given (model, batch)
step launches is decided in one place and can be read off the table below; ``plan`` evaluates it for a step's shapes
(tests/test_routing_gpu.py compares that plan with the kernels a BASELINE.json config's step really launches).

=============================  ===========================================================  =============================
op (key)                       default route                                                 evidence (profiles/)
=============================  ===========================================================  =============================
weight gradient dW = dYᵀX      csrc/gemm_w4.hip weight-gradient mode (K split over           r5_wgrad_w4_ab.txt
                               workgroups, fp32 slabs + csrc/gemm.hip split-K pass) from
                               ``wgrad_min_rows`` (4096) token rows; hipBLASLt below (a       r6_wgrad_small_rows.txt
                               256x256-tile kernel has ~23 us of fixed cost); deferred over
                               a GA window (ops/gemm.py WgradDefer)                          r5_defer_wgrad_ab.txt
projection forward             hipBLASLt + TunableOp table (``proj_fwd`` = lib); arms:       r6_proj_fwd_arms_ab.txt,
Y = X Wᵀ (+ b)                 ``narrow`` (w4 for K <= 1024, N <= 4096 at >=                 r6_w4_vs_lib_nt_pmc.txt
                               ``proj_fwd_min_rows`` tokens: step-neutral), ``w4`` (every
                               forward: -0.46 % t5-base, -0.67 % bart-large)
projection input gradient      w4 from ``proj_dgrad_min_rows`` (16K) token rows at any       r6_dgrad_min_rows_ab.txt,
dX (+)= dY W                   width / depth (early-release schedule: faster than the         r6_dgrad_rows_ab.txt
                               library on every such shape); hipBLASLt below (``proj_dgrad``
                               = rows)
FFN, ReLU (T5)                 forward: w4 ReLU + row-Weyl dropout + bit-mask epilogue at     r6_ffn_rowweyl_dropout_ab.txt,
                               every fused size (``ffn_w4_min_rows`` = 0; the ping-pong       r6_ffn_w4_rows_ab.txt
                               forward below it is the A/B arm); backward: w4 through the
                               bit mask; < ``ffn_min_rows`` (1025) rows: hipBLASLt +
                               csrc/act.hip (unfused)                                        r5_ffn_small_rows_ab.txt
FFN, GELU (BART)               ping-pong GEMM with GELU epilogues (``ffn_gelu`` = pp; w4      r5_w4_gelu_ab.txt
                               GELU epilogues measured 0.25-0.43 % slower)
FFN, gated GELU (FLAN-T5)      one GEMM pairing gate / up columns when tokens x d_ff >=       r4_gemm_pp_stage_ab.txt
                               ``gated_min_mf`` and d_model <= ``gated_max_d`` (1024)
LM head + cross-entropy        full logits while they fit ``lmhead_full_mb`` (16 GiB),       r3_lmhead_b512_ab.txt,
                               else vocabulary chunks of ``lmhead_chunk_mb``; the fused       r4_lmhead_fused_ab.txt,
                               GEMM+CE (w4 CEF / CEB epilogues) when ``lmhead`` = fused or    r5_bart_lmhead_fused_ab.txt
                               (auto) when the logits would exceed the budget
attention                      csrc/attn.hip bf16 flash kernels; fp32 inputs on the fp32      r4_t5base_fp32_b16_summary.txt
                               MFMA kernels of csrc/attn_f32.hip (``attn_f32`` = 1)
long-context attention         query chunks of ``attn_chunk`` rows from ``attn_chunk_min``   (parallel/context.py)
weight gradients, small        side stream for micro-batches <= ``wgrad_stream_max_tokens``  r4_wgrad_stream_ab.txt
micro-batches                  (``wgrad_stream`` = auto | 1 | 0)
beam search                    fused device-side beam step (``gen_fused_beam``), encoder K/V  r3_eval_beam_fused.jsonl
                               shared by a batch entry's beams (``gen_shared_cross``)
gradient reducer               native C++ engine (``reducer`` = native | python), buckets     r5_gloo2_gpu.txt
                               re-laid in gradient-ready order (``rebuild_buckets``)
HIP-graph DP schedule          overlap: backward segments cut at bucket readiness            r5_gloo2_gpu_final.txt
                               (``graph_comm`` = overlap | split | capture)
=============================  ===========================================================  =============================

Fixed choices that used to be switches (their losing arms were deleted in round 6): the ReLU backward reads the
forward's bit mask; GELU / attention / post-LN bias gradients come from the producing kernel's column partials; the
post-LN residual gradient accumulates in the input-gradient GEMM (beta = 1); the ping-pong kernel persists on every
shape it serves; the T5 attention forward adds saturated bias tiles as scalars.

Overrides (A/B runs, tests): ``DLLM_ROUTE="key=value,key=value"`` (read at every ``get``: a test may change it between
calls); unknown keys fail loudly.
"""
from __future__ import annotations

import os

DEFAULTS: dict = {
    # projection GEMMs (ops/gemm.py)
    "proj_fwd": "lib",            # lib | w4 | narrow (w4 for K <= 1024, N <= 4096 at >= proj_fwd_min_rows tokens)
    "proj_fwd_min_rows": 131072,
    "proj_dgrad": "rows",         # rows | w4 | lib
    "proj_dgrad_min_rows": 16384,
    # weight gradients (ops/gemm.py): w4 weight-gradient mode from this many token rows, hipBLASLt (fp32 addmm) below
    "wgrad_min_rows": 4096,
    # feed-forward blocks (ops/ffn.py)
    "ffn": "fused",               # fused | unfused
    "ffn_min_rows": 1025,
    "ffn_w4_min_rows": 0,
    "ffn_gelu": "pp",             # pp | w4
    "gated_min_mf": 2 * 256 * 256 * 256,
    "gated_max_d": 1024,
    # LM head + cross-entropy (ops/lm_head.py)
    "lmhead": "auto",             # auto | fused | logits
    "lmhead_full_mb": 16384.0,
    "lmhead_chunk_mb": 128.0,
    # attention (ops/attention.py, parallel/context.py)
    "attn_f32": 1,
    "attn_chunk": 0,              # 0: 8192 rows for < 32 rows per head, else 4096
    "attn_chunk_min": 8192,
    # weight-gradient side stream (ops/streams.py)
    "wgrad_stream": "auto",       # auto | 1 | 0
    "wgrad_stream_max_tokens": 32768,
    "wgrad_stream_lag": 2,
    "wgrad_stream_sites": "",     # comma list of layer roles ("" = the default pairing policy)
    # generation (models/generation.py)
    "gen_fused_beam": 1,
    "gen_shared_cross": 1,
    "gen_check_every": 8,
    "gen_host": 0,
    # data-parallel runtime (parallel/reducer.py, train/graph.py)
    "reducer": "native",          # native | python
    "rebuild_buckets": 1,
    "graph_comm": "",             # "" = overlap when the reducer overlaps, else split
    # evaluation batch on the GPU (cli.py)
    "eval_batch": 256,
    # read by the C++ launchers (csrc/route.h): ping-pong GEMM tile-group size; test hook forcing the short-query
    # dK/dV kernel on any launch size
    "gemm_grp": 4,
    "attn_dkdv_sq_force": 0,
    # csrc/gemm_w4.hip k-loop schedule (template RS): 769 = early fragment reads + DMAs riding on MFMAs + the LDS buffer
    # released half-way through sub-step 0 so the next DMA spreads over 88 MFMAs (default); 257 = without the early
    # release, 1 = the round-5 schedule; bits 16-128 = timing ablations (tools/gemm_w4_bench.py --ablate; garbage)
    "w4_sched": 769,
}

_cache: tuple[str, dict] | None = None


def overrides() -> dict:
    """The parsed ``DLLM_ROUTE`` overrides (typed like their defaults)."""
    global _cache
    raw = os.environ.get("DLLM_ROUTE", "")
    if _cache is not None and _cache[0] == raw:
        return _cache[1]
    out = {}
    for item in filter(None, (x.strip() for x in raw.split(","))):
        k, _, v = item.partition("=")
        k = k.strip()
        if k not in DEFAULTS:
            raise KeyError(f"DLLM_ROUTE: unknown key {k!r} (known: {', '.join(sorted(DEFAULTS))})")
        d = DEFAULTS[k]
        out[k] = type(d)(float(v)) if isinstance(d, (int, float)) and not isinstance(d, bool) else v.strip()
    _cache = (raw, out)
    return out


def merged(**kw) -> str:
    """A ``DLLM_ROUTE`` string: the current overrides with ``kw`` added (tests: ``monkeypatch.setenv("DLLM_ROUTE",
    routing.merged(lmhead="fused"))``)."""
    cur = dict(overrides())
    for k, v in kw.items():
        if k not in DEFAULTS:
            raise KeyError(f"unknown route key {k!r}")
        cur[k] = v
    return ",".join(f"{k}={v}" for k, v in cur.items())


def get(key: str):
    """The route / threshold ``key`` of the table (``DLLM_ROUTE`` override, else its default)."""
    ov = overrides()
    return ov[key] if key in ov else DEFAULTS[key]


def plan(model: str, tokens_enc: int, tokens_dec: int, d_model: int, d_ff: int, act: str, vocab: int) -> dict:
    """What the table routes for one training step of an encoder-decoder model with these shapes (per micro-batch
    token rows): a dict op -> kernel family, as the tests and docs/ARCHITECTURE.md read it."""
    rows = {"enc": tokens_enc, "dec": tokens_dec}
    out = {}
    dmode = get("proj_dgrad")
    for side, r in rows.items():
        out[f"{side}.wgrad"] = "w4-wgrad" if r >= get("wgrad_min_rows") else "hipblaslt"
        fm = get("proj_fwd")
        out[f"{side}.proj_fwd"] = ("w4" if fm == "w4" else "w4-narrow" if fm == "narrow" and r >= get("proj_fwd_min_rows")
                                   else "hipblaslt")
        if dmode == "w4":
            dg = "w4"
        elif dmode == "lib":
            dg = "hipblaslt"
        else:
            dg = "w4" if r >= get("proj_dgrad_min_rows") else "hipblaslt"
        out[f"{side}.proj_dgrad"] = dg
        if get("ffn") != "fused" or r < get("ffn_min_rows"):
            out[f"{side}.ffn"] = "hipblaslt+act"
        elif act == "relu":
            out[f"{side}.ffn"] = "w4-relu" if r >= get("ffn_w4_min_rows") else "pingpong-relu+w4-drelu"
        elif act in ("gelu", "gelu_new", "gelu_fast") and not act.startswith("gated"):
            out[f"{side}.ffn"] = "w4-gelu" if get("ffn_gelu") == "w4" else "pingpong-gelu"
        else:
            out[f"{side}.ffn"] = ("pingpong-geglu" if r * d_ff >= get("gated_min_mf") and d_model <= get("gated_max_d")
                                  else "hipblaslt+act")
    logits_mb = tokens_dec * vocab * 2 / 2**20
    lm = get("lmhead")
    out["lm_head"] = ("w4-fused-ce" if lm == "fused" or (lm == "auto" and logits_mb > get("lmhead_full_mb"))
                      else "hipblaslt+ce")
    out["attention"] = "attn.hip"
    return out
