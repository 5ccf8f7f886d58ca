"""Decode the C2 batch's JSON v2 (or proto3) encoding on the device a few times (for rocprofv3
--stats / --pmc of the k_js_* or k_proto3_* kernels):
python tools/json_decode_run.py [--traces N] [--reps R] [--format json|proto3]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--traces", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--format", default="json", choices=["json", "proto3"])
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime first, as the tests do)
    from zipkin_amd import synth
    from zipkin_amd.columnar import Dictionary
    from zipkin_amd.jsonv2 import JsonV2Decoder
    w = synth.C2.scaled(a.traces)
    cols = synth.generate(w)
    if a.format == "proto3":
        from zipkin_amd.proto3 import Proto3Decoder
        data = synth.encode_proto3(cols, synth.service_names(w)).tobytes()
        dec = Proto3Decoder(Dictionary(), Dictionary(), Dictionary())
    else:
        data = synth.encode_json_v2(cols, synth.service_names(w)).tobytes()
        dec = JsonV2Decoder(Dictionary(), Dictionary(), Dictionary())
    for i in range(a.reps):
        t0 = time.perf_counter()
        b = dec.decode(data)
        dt = (time.perf_counter() - t0) * 1e3
        if a.format == "proto3":
            print(f"rep {i}: {b.n_spans} spans, {len(data) / 1e9:.2f} GB, kernel {dec._dec.kernel_ms():.2f} ms, "
                  f"call {dt:.1f} ms", flush=True)
        else:
            print(f"rep {i}: {b.n_spans} spans, {len(data) / 1e9:.2f} GB, structure {dec.struct_ms():.2f} ms, "
                  f"spans {dec.kernel_ms():.2f} ms ({dec.exact_spans()} exact), call {dt:.1f} ms", flush=True)
    dec.close()


if __name__ == "__main__":
    main()
