#!/usr/bin/env python3
"""bench.py -- audio samples/s for the RWKV-TTS hot path on MI355X (BASELINE.json metric).

One "step" = one full batch of B=32 synthetic requests through the hot path on each GPU
(config 3 of BASELINE.json): 32-token prompt -> RWKV-7 0.4B prefill -> 32 global tokens ->
TAG_1 -> 512 semantic tokens (fixed-length benchmark mode, EOS masked) with the exact
device sampler, continuous batching in 32 GPU slots. Weights are random-init bf16 of the assumed
0.4B architecture (no checkpoints offline), broadcast from rank 0 over RCCL. value = all ranks'
audio samples (320 per semantic token @16 kHz) / max-over-ranks wall time. Each step ends with the
BiCodec decoder (HIP MFMA conv stack, assumed SparkTTS dims, random-init weights) turning every
request's 32 global + 512 semantic tokens into PCM, so the timed region is tokens -> waveform.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]. N > 1 runs one process per GPU:
under torch.distributed.run (RANK / WORLD_SIZE set by the launcher), or, when WORLD_SIZE is unset,
bench.py starts the N ranks itself (before anything touches a GPU) and relays rank 0's line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))

import numpy as np  # noqa: E402

B_PER_GPU = 32
PROMPT_TEXT = 24
SEMANTIC = 512
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA


def codec_flops(cd, T):
    """Algorithmic FLOPs (2 per multiply-add, f32-equivalent) of the BiCodec decoder for T
    frames, by profiling class: the bf16 hi+lo split doubles MFMA work but not
    this count."""
    L, P, I, C = cd["latent_dim"], cd["prenet_dim"], cd["prenet_inter"], cd["dec_channels"]
    f = {"codec_prenet_gemm": 2 * T * (L * P + 7 * P * P + cd["prenet_layers"] * 2 * P * I + P * L),
         "codec_conv_in": 2 * T * 7 * L * C}
    m = 1
    for i in range(cd["n_up"]):
        s, K, Co = cd["up_rates"][i], cd["up_kernels"][i], C // 2
        f[f"codec_convT@{Co}"] = 2 * T * m * C * Co * K
        m *= s
        f[f"codec_res_conv7@{Co}"] = 3 * 2 * T * m * 7 * Co * Co
        f[f"codec_res_conv1@{Co}"] = 3 * 2 * T * m * Co * Co
        # residual units fused into one launch each (codec.hip resunit_fused, 96 channels)
        f[f"codec_resunit@{Co}"] = f[f"codec_res_conv7@{Co}"] + f[f"codec_res_conv1@{Co}"]
        C = Co
    return f


def _file_build(path):
    """The build id a profile summary was measured on (tools/: "build" in the JSON summaries, a
    "# build <id>" first line in the text ones), or None for summaries made before round 6."""
    try:
        if path.endswith(".json"):
            return json.load(open(path)).get("build")
        with open(path) as f:
            first = f.readline().split()
        return first[2] if len(first) == 3 and first[:2] == ["#", "build"] else None
    except (OSError, ValueError):
        return None


def profile_summary(pattern):
    """The committed profile summary (profiles/<pattern>) measured on THIS library build: the one whose
    build id (rwkvtts._ffi.build_id(), a hash of the library's sources) equals the running tree's;
    several: the newest name. None matching: the newest name, flagged (build_match False) -- never
    picked by name order alone (lexicographic order had picked another build's)."""
    import glob
    from rwkvtts import _ffi
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    if not files:
        return None, False
    bid = _ffi.build_id()
    match = [f for f in files if _file_build(f) == bid]
    return (match[-1], True) if match else (max(files, key=os.path.getmtime), False)


def pmc_traffic(kernel):
    """HBM bytes per launch of a decode-step kernel from the PMC summary of this build
    (profiles/rNN_pmc_traffic.json, made by tools/gpu_profiles.sh + tools/make_pmc_json.py:
    separate FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled per the gfx950 correction)."""
    f, ok = profile_summary("r*_pmc_traffic.json")
    if not f:
        return None, None, False
    k = json.load(open(f))["kernels"]
    key = kernel if kernel in k else ("ln_mix" if kernel.startswith("ln_mix") else kernel)
    if key not in k:
        return None, None, False
    return k[key]["traffic_bytes"], os.path.relpath(f, ROOT), ok


def mfma_counters(part="codec"):
    """Aggregate MFMA utilisation of the vocoder (or LM) kernels from the counter summary of this
    build (profiles/rNN_mfma_<part>.txt, made by tools/pmc_mfma.sh + tools/mfma_summary.py:
    SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x per-XCD GRBM_GUI_ACTIVE))."""
    import re
    f, ok = profile_summary(f"r*_mfma_{part}.txt")
    if not f:
        return None
    for line in open(f):
        m = re.match(r"TOTAL mfma_util ([0-9.]+) over ([0-9.]+) ms .* ([0-9.]+) TFLOP/s executed", line)
        if m:
            return {"util": float(m.group(1)), "executed_tflops": float(m.group(3)),
                    "source": os.path.relpath(f, ROOT), "build_match": ok}
    return None


def algorithmic_bytes(d, R, head_rows):
    """Per-kernel algorithmic HBM bytes of one decode step with R rows, SURVEY §8d's model (not
    this implementation's intermediates): weights read once, the recurrent state read and
    written once (WKV state H*N*N f32 and the two token-shift vectors C f32 per row and layer),
    plus the embedding rows and the logits of the head rows. Activation planes and split-K
    partial slabs are implementation traffic: they appear in the PMC `traffic`, not here."""
    C, F, L = d["n_embd"], d["n_ffn"], d["n_layer"]
    H, N = C // 64, 64
    Dt = d["d_decay"] + d["d_aaa"] + d["d_mv"] + d["d_gate"]
    per = {
        "gemm_rkv_lora": (3 * C * C + Dt * C) * 2,
        "wkv": R * H * N * N * 4 * 2 + C * Dt * 2,
        "gemm_wo": C * C * 2,
        "gemm_ffn_key": F * C * 2,
        "gemm_ffn_value": C * F * 2,
        "ln_mix_att": R * C * 4 * 2,
        "ln_mix_ffn": R * C * 4 * 2,
    }
    per_step = {k: v * L for k, v in per.items()}
    # the persistent launches of a decode step (k_att_persist / k_ffn_persist) move the bytes of
    # the launches they replace (per launch; not added to per_step again)
    per["att_persist"] = per["ln_mix_att"] + per["gemm_rkv_lora"] + per["wkv"] + per["gemm_wo"]
    per["ffn_persist"] = per["ln_mix_ffn"] + per["gemm_ffn_key"] + per["gemm_ffn_value"]
    per_step["gemm_head"] = head_rows * C * 2 + R * head_rows * 4
    per_step["embed"] = R * C * 2
    return per, per_step


def rocprof_decode(kernel):
    """The kernel's decode-launch statistics from the rocprof trace summary of a bench run on this
    build (profiles/rNN_decode_kernels.json, tools/decode_kernel_summary.py: launches at the
    decode grid only, prefill launches excluded), so the roofline can be recomputed from
    profiles/. Reported beside the live HIP-event figure, never in its place."""
    f, ok = profile_summary("r*_decode_kernels.json")
    if not f:
        return None
    k = json.load(open(f))["kernels"].get(kernel)
    if not k:
        return None
    return {"median_us": k["median_us"], "mean_us": k["mean_us"], "launches": k["launches"],
            "frac_at_median": k.get("frac_at_median"), "source": os.path.relpath(f, ROOT), "build_match": ok}


def batch1_leg(rt, voc, requests, dims):
    """Config 2 of BASELINE.json (the reference's live path: one request at a time on slot 0,
    normal_mode_inference.rs:62-80,222-391): ONE request through the same engine (its R = 1
    decode graphs), timed after a warm-up request; then its PCM by the HIP vocoder (the
    reference keeps ORT-CPU for config 2; there is no ORT here, so the vocoder leg is the GPU
    one and the LM-only rate is reported beside it)."""
    rt.generate_batch(requests(-50)[:1])  # warm-up: captures the one-row graphs
    n_req, t_gen, t_voc, dms, steps, sem = 3, 0.0, 0.0, 0.0, 0, 0
    for k in range(n_req):
        r = requests(-51 - k)[:1]
        t0 = time.perf_counter()
        out = rt.generate_batch(r)
        t_gen += time.perf_counter() - t0
        st = rt.stats()
        dms += st["decode_ms"]
        steps += st["steps"]
        sem += sum(len(s) for _, s in out)
        t1 = time.perf_counter()
        pcm = voc.decode_audio_batch([(g, s) for g, s in out])
        t_voc += time.perf_counter() - t1
        assert sum(p.size for p in pcm) == 320 * sum(len(s) for _, s in out)
    step_ms = dms / max(steps, 1)
    _, per_step = algorithmic_bytes(dims, 1, 8193)
    b = sum(per_step.values())
    samples = 320 * sem
    return {"workload": f"config2: 1 request at a time (B=1), P=32 prompt, 32 global + {SEMANTIC} semantic tokens, "
                        f"exact sampler, HIP vocoder; {n_req} requests timed after one warm-up",
            "samples_per_s": round(samples / (t_gen + t_voc), 1),
            "samples_per_s_lm_only": round(samples / t_gen, 1),
            "rtf": round((t_gen + t_voc) / (samples / 16000.0), 6),
            "ms_per_request": round(1000.0 * (t_gen + t_voc) / n_req, 3),
            "vocoder_ms_per_request": round(1000.0 * t_voc / n_req, 3),
            "decode_steps_per_request": steps // n_req,
            "decode_step_us": round(1000.0 * step_ms, 2),
            "decode_step_roofline": {"bytes_per_step": b, "ms_per_decode_step": round(step_ms, 4),
                                     "achieved": round(b / (step_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                                     "frac": round(b / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--token-chunk-size", type=int, default=2048,
                    help="prompt rows per engine step (all admitted prompts share it; outputs are chunk-invariant, bitwise)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-batch1", action="store_true", help="skip the config-2 (one request) leg")
    ap.add_argument("--voc-delay-ms", type=float, default=0.0,
                    help="start each batch's vocoder this long after its LM finished (pipelining A/B)")
    ap.add_argument("--no-graph-timing", dest="graph_timing", action="store_false",
                    help="per-kernel times from an eager HIP-event pass instead of in-graph stamps")
    ap.add_argument("--profile", action="store_true", help="per-kernel HIP-event pass (default on)")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="run the vocoder of each batch after its LM decode instead of overlapped")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a "
                         "different GPU count than asked for")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import rwkvtts
    from rwkvtts import weights as W

    dims = W.DIMS_04B
    nbytes = W.blob_bytes(dims)
    # ---- weights: synthesised once on rank 0, broadcast over RCCL (xGMI) to every rank
    wdev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    if rank == 0:
        blob = W.synth_blob(dims, seed=20251205)
        wdev.copy_(torch.from_numpy(blob))
        del blob
    from rwkvtts import dist as D
    D.broadcast_blob(wdev, src=0)
    torch.cuda.synchronize()
    rt = rwkvtts.SharedRwkvRuntime(nbytes, device=local, max_slots=B_PER_GPU, token_chunk_size=args.token_chunk_size,
                                   use_graphs=True, device_ptr=wdev.data_ptr())
    del wdev
    # ---- vocoder weights: same scheme (rank 0 synthesises, RCCL broadcast)
    from rwkvtts import codec as CC
    cdims = CC.CODEC_DIMS_FULL
    cw = torch.empty(CC.codec_blob_floats(cdims), dtype=torch.float32, device="cuda")
    if rank == 0:
        cw.copy_(torch.from_numpy(CC.synth_codec_blob(cdims)))
    D.broadcast_blob(cw, src=0)
    voc = CC.BiCodecDetokenizer(cw.cpu().numpy(), cdims, device=local)
    del cw
    torch.cuda.empty_cache()

    def requests(step):
        reqs = []
        for i in range(B_PER_GPU):
            rid = (rank * 1000003 + step * 9176 + i)
            rs = np.random.RandomState(rid % (2**31))
            text = rs.randint(12293, 77822, size=PROMPT_TEXT).tolist()
            props = [77823, 77838, 77869, 77845, 77830, 77826]
            reqs.append(rwkvtts.TtsBatchRequest(text_tokens=text, property_tokens=props,
                                                args=rwkvtts.SamplerArgs(seed=rid, max_tokens=2048),
                                                fixed_semantic=SEMANTIC))
        return reqs

    def run(step):
        out = rt.generate_batch(requests(step))
        pcm = voc.decode_audio_batch([(g, s) for g, s in out])
        n = sum(len(s) for _, s in out)
        assert sum(p.size for p in pcm) == 320 * n, "vocoder output length mismatch"
        return n

    for w in range(args.warmup):
        run(-1 - w)
    # Steps are pipelined the way a server overlaps requests: the vocoder of batch s runs on its
    # own HIP stream (worker thread; ctypes releases the GIL) while the LM decodes batch s + 1.
    # Every batch's PCM is complete inside the timed region.
    from concurrent.futures import ThreadPoolExecutor

    def vocode(out):
        if args.voc_delay_ms > 0:  # start after the next batch's prefill (A/B switch)
            time.sleep(args.voc_delay_ms / 1000.0)
        pcm = voc.decode_audio_batch([(g, s) for g, s in out])
        assert sum(p.size for p in pcm) == 320 * sum(len(s) for _, s in out), "vocoder output length mismatch"
        return len(pcm)

    def pipelined(steps, step0):
        acc = {"gen_ms": 0.0, "decode_ms": 0.0, "prefill_ms": 0.0, "dec_steps": 0, "sem_tokens": 0, "out": None}
        futs = []
        with ThreadPoolExecutor(max_workers=1) as pool:
            for s in range(step0, step0 + steps):
                tg = time.perf_counter()
                out = rt.generate_batch(requests(s))
                acc["gen_ms"] += 1000.0 * (time.perf_counter() - tg)
                acc["sem_tokens"] += sum(len(x) for _, x in out)
                st = rt.stats()
                acc["decode_ms"] += st["decode_ms"]
                acc["prefill_ms"] += st["prefill_ms"]
                acc["dec_steps"] += st["steps"]
                acc["out"] = out
                futs.append(pool.submit(vocode, out) if args.pipeline else None)
                if not args.pipeline:
                    vocode(out)
            for f in futs:
                if f is not None:
                    f.result()
        return acc

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    acc = pipelined(args.steps, 0)  # the timed region: no instrumentation in the decode graphs
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gen_ms, decode_ms, prefill_ms = acc["gen_ms"], acc["decode_ms"], acc["prefill_ms"]
    dec_steps, sem_tokens, out = acc["dec_steps"], acc["sem_tokens"], acc["out"]
    elapsed, total_tokens = D.reduce_run(elapsed, sem_tokens, device="cuda")
    # in-graph kernel timing (rwkvtts_set_profiling mode 2), in a SEPARATE pass after the timed region
    # (ADVICE r4): the decode graphs are recaptured with launch-timeline slots and two more batches
    # run pipelined exactly as timed (the vocoder of each beside the next one's decode); the last step
    # of every decode window is sampled (per launch: first workgroup start -> last workgroup end)
    gprof = {}
    if args.graph_timing and rank == 0:
        rt.set_profiling(2)
        pipelined(2, 10**5)
        gprof = rt.profile()
        rt.set_profiling(0)
    samples = total_tokens * 320
    value = samples / elapsed
    audio_s = samples / 16000.0
    rtf = elapsed / audio_s

    # ---- per-kernel HIP-event pass (same workload, eager launches on the engine's stream)
    roofline = None
    kernels = {}
    step_roof = None
    codec_roof = None
    if rank == 0:
        # decode-step kernels: the in-graph samples of the timed region (the same launches rocprof
        # traces); without them (--no-graph-timing) an eager HIP-event pass of one batch. The
        # vocoder's own pass runs alone.
        if gprof:
            prof = gprof
            prof_out = out
        else:
            rt.set_profiling(True)
            prof_out = rt.generate_batch(requests(10**6))
            prof = rt.profile()
            rt.set_profiling(False)
        voc.set_profiling(True)
        vocode(prof_out)
        vprof = voc.profile()
        voc.set_profiling(False)
        st = rt.stats()
        R = B_PER_GPU
        per_launch, per_step = algorithmic_bytes(dims, R, 8193)
        for name, (launches, ms) in prof.items():
            kernels[name] = {"launches": launches, "avg_us": 1000.0 * ms / max(launches, 1), "total_ms": ms}
        # dominant kernel by total time among the decode-step kernels with a byte model (launched
        # at least once per decode step: prefill-only launches are not the decode loop's)
        n_dec = max((v["launches"] for v in kernels.values()), default=0)
        cand = [(v["total_ms"], k) for k, v in kernels.items() if k in per_launch and v["launches"] * 4 >= n_dec]
        if cand:
            _, dom = max(cand)
            avg_s = kernels[dom]["avg_us"] * 1e-6
            ach = per_launch[dom] / avg_s / 1e9
            traffic, tsrc, tok = pmc_traffic(dom)
            roofline = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_source": tsrc, "traffic_build_match": tok, "build": rwkvtts._ffi.build_id(),
                        "bytes_per_launch": per_launch[dom],
                        "avg_us": round(kernels[dom]["avg_us"], 2),
                        "avg_us_source": ("in-graph launch stamps of a separate pass after the timed region (2 "
                                          "batches pipelined as timed, the vocoder beside the decode; last step of "
                                          "every decode window: first workgroup start -> last workgroup end)"
                                          if gprof else "HIP events on the engine stream, eager launches (one batch)"),
                        "rocprof": rocprof_decode(dom)}
        # vocoder: MFMA-bound conv stack, achieved TFLOP/s per class and for the whole decoder
        cfl = codec_flops(cdims, B_PER_GPU * SEMANTIC)
        cfl_total = sum(v for k, v in cfl.items() if not k.startswith("codec_resunit"))  # fused = conv7 + conv1
        vk = {}
        for name, (launches, ms) in vprof.items():
            e = {"launches": launches, "avg_us": round(1000.0 * ms / max(launches, 1), 2), "total_ms": round(ms, 3)}
            if name in cfl and ms > 0:
                e["tflops"] = round(cfl[name] / (ms * 1e-3) / 1e12, 1)
            vk[name] = e
        vtot = sum(ms for _, ms in vprof.values())
        codec_roof = {"bound": "mfma", "flops_per_batch": cfl_total, "ms_per_batch": round(vtot, 3),
                      "achieved": round(cfl_total / (vtot * 1e-3) / 1e12, 1),
                      "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                      "frac": round(cfl_total / (vtot * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4),
                      "mfma_counters": mfma_counters("codec"),
                      "kernels": vk}
        # whole decode step (graph-replayed timing from the timed region)
        if dec_steps:
            step_ms = decode_ms / dec_steps
            step_bytes = sum(per_step.values())
            step_roof = {"bytes_per_step": step_bytes, "ms_per_decode_step": round(step_ms, 4),
                         "achieved": round(step_bytes / (step_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                         "frac": round(step_bytes / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}

    b1 = batch1_leg(rt, voc, requests, dims) if rank == 0 and not args.no_batch1 else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(dims, cdims, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "audio samples/sec (16 kHz) for RWKV-TTS 0.4B, batch=32 per GPU",
            "value": round(value, 1), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random-init bf16 weights of the assumed 0.4B RWKV-7 arch, synthetic prompts)",
            "rtf": round(rtf, 6),
            "config": {"workload": "config3: 32 requests/GPU, P=32 prompt, 32 global + 512 semantic tokens, "
                                   "exact sampler, + BiCodec vocoder -> PCM (vocoder of batch s overlapped with LM of batch s+1 on its own stream)",
                       "global_batch": B_PER_GPU * world, "seq_len": 32 + 33 + SEMANTIC,
                       "parallelism": f"dp{world} (request sharding)"},
            # where a step's wall time goes (rank 0, per batch): generate_batch wall time, of it
            # the engine's decode / prefill stream time; the rest of ms_per_step is the last
            # batch's vocoder (not overlapped) spread over the steps
            "breakdown_ms_per_batch": {"generate": round(gen_ms / args.steps, 3),
                                       "decode": round(decode_ms / args.steps, 3),
                                       "prefill": round(prefill_ms / args.steps, 3),
                                       "decode_steps": dec_steps // max(1, args.steps)},
            "roofline": roofline,
            "decode_step_roofline": step_roof,
            "batch1": b1,
            "codec_roofline": codec_roof,
            "kernels": kernels,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    rt.close()
    voc.close()
    if world > 1:
        dist.destroy_process_group()


def spawn_ranks(n):
    """--gpus N without a launcher: start ranks 0..N-1 as child processes (this process never
    touches a GPU), rendezvous on 127.0.0.1, and exit with the first non-zero child status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        c = p.wait()
        rc = rc or c
    return rc


def host_cpu():
    """nproc and the CPU model of this host (lscpu 'Model name')."""
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return os.cpu_count(), model


def cpu_baseline(dims, cdims, seconds):
    """The oracle (C restatement of the reference path: fp16-stored weights, f32 math -- web-rwkv's
    Bundle<f32> numerics -- 1 request, sequential like process_batch_with_independent_contexts)
    built here with -O3 -march=native (the reference builds with target-cpu=native,
    .cargo/config.toml:2) and run with OpenMP on this process's CPU share (OMP_NUM_THREADS, else
    every core), timed on a bounded sample of the same request and extrapolated to the full
    request (P + 33 + S - 1 forwards -> 320*S samples), plus the oracle vocoder timed on a
    16-frame utterance and scaled linearly to S frames (convolutions are linear in T)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from rwkvtts import _ffi
    from rwkvtts import weights as W
    oracle.use_native()
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    oracle.lib().oracle_set_threads(cores)
    nproc, model = host_cpu()
    blob = W.synth_blob(dims, seed=20251205, dtype=_ffi.DTYPE_F16)
    om = oracle.Model(blob)
    del blob
    st = om.new_state()
    toks = [77823, 77838, 77869, 77845, 77830, 77826, 8195] + list(range(20000, 20024)) + [8193]
    t0 = time.perf_counter()
    n = 0
    while True:
        tok = toks[n] if n < len(toks) else 8196 + (n % 4096)
        om.forward(st, tok, 4096 if n >= len(toks) - 1 else 0)
        n += 1
        if time.perf_counter() - t0 > seconds or n >= 2000:
            break
    per_fwd = (time.perf_counter() - t0) / n
    fwd_per_req = 32 + 33 + SEMANTIC - 1
    del om
    from rwkvtts import codec as CC
    cw = CC.synth_codec_blob(cdims)
    Tc = 16
    rs = np.random.default_rng(0)
    t1 = time.perf_counter()
    oracle.codec_decode(CC.make_codec_dims(cdims), cw, rs.integers(0, 8192, Tc), rs.integers(0, 4096, 32))
    voc_s = (time.perf_counter() - t1) * SEMANTIC / Tc
    val = 320 * SEMANTIC / (fwd_per_req * per_fwd + voc_s)
    return {"value": round(val, 1), "unit": "samples/s", "cores": cores, "kind": "port",
            "host": {"nproc": nproc, "model": model, "build": "gcc -O3 -march=native -fopenmp"},
            "sample": f"oracle f32 RWKV-7 forward on fp16 weights, 1 request, {n} forwards timed "
                      f"({per_fwd*1e3:.1f} ms each), "
                      f"extrapolated to {fwd_per_req} forwards; oracle vocoder on {Tc} frames scaled to "
                      f"{SEMANTIC} ({voc_s:.2f} s); {320*SEMANTIC} samples per request"}


if __name__ == "__main__":
    main()
