"""A/B timing of attention builds in ONE process (cdna_hip_programming.md §5.4 rule 24: compare variants side by
side, interleaved, not across boxes).

  python tools/attn_ab.py build NAME [hipcc flags...]   -> tools/_ab/NAME.so (attention.hip + errors.hip)
  python tools/attn_ab.py run NAME1 NAME2 ...           -> per shape: fwd / bwd median us and TF of every build,
                                                           plus max |diff| of each build's outputs vs the first
"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
OUT = os.environ.get("AB_DIR", os.path.join(HERE, "_ab"))  # AB_DIR=ab_builds: builds that travel to the GPU box
CSRC = os.path.join(ROOT, "simlingo_amd", "csrc")


def build(name, flags):
    """SRC=path overrides the attention source (e.g. a `git show HEAD:...` copy under tools/_ab/)."""
    os.makedirs(OUT, exist_ok=True)
    src = os.environ.get("SRC", os.path.join(CSRC, "attention.hip"))
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
           "-munsafe-fp-atomics", f"-I{ROOT}/include", f"-I{CSRC}", *flags,
           src, os.path.join(CSRC, "errors.hip"), "-o", os.path.join(OUT, name + ".so")]
    subprocess.run(cmd, check=True)
    print("built", name, flags)


def run(names):
    import torch
    from simlingo_amd import kernels as K
    dev = torch.device("cuda")
    libs = [ctypes.CDLL(os.path.join(OUT, n + ".so"), mode=ctypes.RTLD_LOCAL) for n in names]
    shapes = {"vit": dict(B=16, S=1025, Hq=16, Hkv=16, causal=False), "llm": dict(B=8, S=798, Hq=14, Hkv=2, causal=True)}
    for sname, c in shapes.items():
        B, S, Hq, Hkv = c["B"], c["S"], c["Hq"], c["Hkv"]
        torch.manual_seed(0)
        qkv = (torch.randn(B * S, (Hq + 2 * Hkv) * 64, device=dev) * 0.5).bfloat16()
        q, k, v = qkv[:, :Hq * 64], qkv[:, Hq * 64:(Hq + Hkv) * 64], qkv[:, (Hq + Hkv) * 64:]
        kw = dict(B=B, S=S, Hq=Hq, Hkv=Hkv, causal=c["causal"])
        if c["causal"]:
            kw["seqlens"] = torch.full((B,), S, dtype=torch.int32, device=dev)
        fl = 4.0 * B * Hq * S * S * 64 * (0.5 if c["causal"] else 1.0)
        dout = torch.randn(B * S, Hq * 64, device=dev).bfloat16()
        outs, times = [], [[[], []] for _ in libs]
        st = K.stream_ptr()
        for rep in range(7):
            for j, lib in enumerate(libs):
                o = torch.empty(B * S, Hq * 64, device=dev, dtype=torch.bfloat16)
                lse = torch.empty(B * Hq * S, device=dev)
                d = K.attn_desc(q, k, v, o, lse, **kw)
                dqkv = torch.zeros_like(qkv)
                ws = K.attn_ws(B, S, Hq, Hkv, dev)
                g = K.AttnBwdDesc()
                g.dout, g.lddo = dout.data_ptr(), dout.stride(0)
                dq, dk, dv = dqkv[:, :Hq * 64], dqkv[:, Hq * 64:(Hq + Hkv) * 64], dqkv[:, (Hq + Hkv) * 64:]
                g.dq, g.lddq, g.dk, g.lddk, g.dv, g.lddv = dq.data_ptr(), dq.stride(0), dk.data_ptr(), dk.stride(0), \
                    dv.data_ptr(), dv.stride(0)
                g.delta_ws, g.dq_acc = ws["delta"].data_ptr(), ws["dq_acc"].data_ptr()
                g.dk_acc = ws["dk_acc"].data_ptr() if "dk_acc" in ws else 0
                g.dv_acc = ws["dv_acc"].data_ptr() if "dv_acc" in ws else 0
                for which, fn in ((0, lambda: lib.slx_attn_fwd(ctypes.byref(d), st)),
                                  (1, lambda: lib.slx_attn_bwd(ctypes.byref(d), ctypes.byref(g), st))):
                    fn()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(10):
                        rc = fn()
                    e1.record()
                    torch.cuda.synchronize()
                    assert rc == 0, rc
                    times[j][which].append(e0.elapsed_time(e1) / 10)
                if rep == 0:
                    outs.append((o.float(), dqkv.float()))
        for j, n in enumerate(names):
            tf, tb = sorted(times[j][0])[3], sorted(times[j][1])[3]
            do = (outs[j][0] - outs[0][0]).abs().max().item()
            dg = (outs[j][1] - outs[0][1]).abs().max().item()
            print(f"{sname} {n:>12}: fwd {tf * 1e3:7.1f} us {fl / tf / 1e9:6.0f} TF | bwd {tb * 1e3:7.1f} us "
                  f"{2.5 * fl / tb / 1e9:6.0f} TF | vs {names[0]}: o {do:.2e} dqkv {dg:.2e}", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2], sys.argv[3:])
    else:
        run(sys.argv[2:])
