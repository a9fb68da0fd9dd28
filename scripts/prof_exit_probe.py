#!/usr/bin/env python3
"""Process-exit probe for rocprofv3 teardown crashes.

    rocprofv3 --kernel-trace -d gpurun_out/<dir> -o run --output-format csv -- \
        python scripts/prof_exit_probe.py cumask|coop|plain

cumask: a kernel on a CU-masked stream (its own hardware queue), then exit;
coop:   the one-launch cooperative l-bfgs fit (lsq_qn.hip), its result read, then exit;
coopreset: coop, then hipDeviceReset() before interpreter exit (the runtime's queues -- the
        cooperative-launch queue among them -- destroyed while the profiler is still attached);
plain:  the same work on the default stream only (control).
Prints "probe done" before interpreter exit: a crash after that line is a teardown crash."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from net.jgp.labs.sparkdq4ml_amd.ops import device, kernels, native

    mode = sys.argv[1]
    h = native.hip()
    x = torch.randn(1 << 20, device="cuda")
    if mode == "cumask":
        from net.jgp.labs.sparkdq4ml_amd.runtime import streams

        cus = device._cus(h)
        st = streams.cu_masked_stream(list(range(cus)), cus, torch.device("cuda", 0), tag=7)
        with torch.cuda.stream(st):
            y = (x * 2.0).sum()
        st.synchronize()
        print("sum", float(y))
    elif mode in ("coop", "coopreset"):
        d, n = 512, 100_000
        X = torch.randn(d, n, device="cuda")
        y = torch.linspace(-1, 1, d, device="cuda") @ X + 0.5
        T = device.pack_wide([X.to(torch.bfloat16)], 16, None)
        P = kernels.lsq_passes(T, y.double(), None, None)
        head = torch.cat([P.scalars(), P.moments()])
        out = P.qn_fit(head, True, True, 0.01, 0.0, 50, 1e-9)
        print("qn status", int(out[d + 1].item()), "evals", int(out[d + 5].item()))
    else:
        print("sum", float((x * 2.0).sum()))
    torch.cuda.synchronize()
    if mode == "coopreset":
        import ctypes

        rc = ctypes.CDLL("libamdhip64.so").hipDeviceReset()
        print("hipDeviceReset", rc, flush=True)
    if os.environ.get("PROBE_MAPS"):  # the process map, to place the crash's PCs in their libraries
        with open("/proc/self/maps") as f, open(os.environ["PROBE_MAPS"], "w") as o:
            o.write(f.read())
    print("probe done", flush=True)


if __name__ == "__main__":
    main()
