"""HBM traffic of the roofline kernel (bench.py `roofline.traffic`), measured with rocprofv3 PMC counters.

  run   --config vla|base [--calls N]   : issue N copies of exactly the bench's FC1 call (same K.mm call site,
                                          shapes, epilogue and operands as engine.py / base_engine.py) on cuda:0
  parse --config vla|base --fetch DIR --write DIR --out FILE
                                        : per-call HBM bytes from two separate rocprofv3 passes
                                          (--pmc FETCH_SIZE, then --pmc WRITE_SIZE; they cannot share a pass)

Units and gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are KiB; on gfx950
FETCH_SIZE tallies exactly half the bytes of wide (16 B/lane) coalesced reads — global_load and buffer_load..lds
alike, which is how the GEMM streams A and B — so reads are doubled; WRITE_SIZE is exact for 16-B stores.
A call may be more than one dispatch (the M-remainder peel): every gemm_bf16 dispatch of the process is
summed and divided by the number of calls.
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {  # M = images x tokens, N = FFN, K = width (bench.py probe shapes)
    "vla": dict(M=16 * 1025, N=4096, K=1024, epi="GELU", tag="vla_b8"),
    "base": dict(M=64 * 577, N=4096, K=1024, epi="QGELU", tag="base_b32"),
    # the VLA step's dominant kernel: the InternViT fc2.w + fc1.w weight-gradient pair (engine.py "vit.wgrad_fc"),
    # one slx_gemm_bf16_pair launch of two accumulating TN GEMMs with K = tokens; recorded as the "_pair" record
    "vla_pair": dict(M=16 * 1025, N=4096, K=1024, epi="PAIR", tag="vla_b8_pair"),
}


def algorithmic_bytes(s):
    if s["epi"] == "PAIR":  # dY, GELU output, dH, LN2 output (bf16) read once; both f32 dW read + written
        return s["M"] * 2 * (2 * s["K"] + 2 * s["N"]) + 2 * 2 * 4 * s["N"] * s["K"]
    # A [M,K] bf16 + W [N,K] bf16 + bias f32 read; activation [M,N] bf16 + pre-activation aux [M,N] bf16 written
    return 2 * s["M"] * s["K"] + 2 * s["N"] * s["K"] + 4 * s["N"] + 2 * 2 * s["M"] * s["N"]


def run(cfg, calls):
    import torch
    from simlingo_amd import kernels as K
    s = SHAPES[cfg]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    if s["epi"] == "PAIR":  # exactly engine.py's mm_pair call: (g, hact, dW_fc2), (dh, h2, dW_fc1), TN, accumulate
        M, N, D = s["M"], s["N"], s["K"]
        gy = (torch.randn(M, D, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        hact = (torch.randn(M, N, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        dh = (torch.randn(M, N, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        h2 = (torch.randn(M, D, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        dw2 = torch.zeros(D, N, device=dev)
        dw1 = torch.zeros(N, D, device=dev)
        torch.cuda.synchronize()
        for _ in range(calls):
            K.mm_pair((gy, hact, dw2), (dh, h2, dw1))
        torch.cuda.synchronize()
        print(json.dumps({"config": cfg, "calls": calls, **s}))
        return
    x = (torch.randn(s["M"], s["K"], device=dev, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(s["N"], s["K"], device=dev, generator=g) * 0.03).to(torch.bfloat16)
    b = torch.randn(s["N"], device=dev, generator=g) * 0.1
    act = torch.empty(s["M"], s["N"], dtype=torch.bfloat16, device=dev)
    pre = torch.empty_like(act)
    epi = getattr(K, "EPI_" + s["epi"])
    torch.cuda.synchronize()
    for _ in range(calls):
        K.mm(x, w, act, bias=b, epi=epi, aux_out=pre, ldaux_out=s["N"])
    torch.cuda.synchronize()
    print(json.dumps({"config": cfg, "calls": calls, **s}))


def _sum_counter(d, name, regex="gemm_bf16"):
    import re
    tot, n = 0.0, 0
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if row.get("Counter_Name") != name or not re.search(regex, row.get("Kernel_Name", "")):
                continue
            tot += float(row["Counter_Value"])
            n += 1
    return tot, n


def parse(cfg, fetch_dir, write_dir, calls, out):
    s = SHAPES[cfg]
    f_kib, nf = _sum_counter(fetch_dir, "FETCH_SIZE")
    w_kib, nw = _sum_counter(write_dir, "WRITE_SIZE")
    if not nf or not nw:
        raise SystemExit(f"no gemm_bf16 dispatches with counters (fetch {nf}, write {nw})")
    rd = 2.0 * f_kib * 1024 / calls
    wr = w_kib * 1024 / calls
    alg = algorithmic_bytes(s)
    rec = {"config": cfg, "M": s["M"], "N": s["N"], "K": s["K"], "epilogue": s["epi"], "calls": calls,
           "dispatches_per_call": nf / calls, "read_bytes": rd, "write_bytes": wr, "traffic_bytes": rd + wr,
           "algorithmic_bytes": alg, "traffic_over_algorithmic": round((rd + wr) / alg, 3),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; KiB -> bytes; "
                     "FETCH_SIZE x2 (gfx950 half-count of 16-B/lane reads); summed over the call's dispatches"}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "parse"])
    ap.add_argument("--config", default="vla", choices=sorted(SHAPES))
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.mode == "run":
        run(a.config, a.calls)
    else:
        parse(a.config, a.fetch, a.write, a.calls, a.out)
