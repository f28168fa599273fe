"""Builds the timing-only phase probes of agg_w32 that tools/aggw_probe.sh runs
(run here, on the CPU, after the default build): libpinsage_hip_p1.so drops the
projection's k loop, libpinsage_hip_p2.so the self-row copy and the aggregation.
Their results are wrong by construction; they only time the remaining phases."""
import glob
import os
import subprocess

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gcn-song-embeddings_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def probe_source():
    s = open(os.path.join(CSRC, "aggw.hip")).read()
    k = s.index("__global__ __launch_bounds__(kAw32Threads) void agg_w32_kernel(")
    head, tail = s[:k], s[k:]
    for old, new in [
        ("    // ---- self rows -> A[:, 0:d)\n    {", "    // ---- self rows -> A[:, 0:d)\n    if (PS_AGGW_PROBE != 2) {"),
        ("    // ---- aggregate -> A[:, d:K) and agg (thread: row tid / 32, float4 columns\n"
         "    //      (tid % 32) + 32 j); four slots' rows in flight per round\n    {",
         "    // ---- aggregate\n    if (PS_AGGW_PROBE != 2) {"),
        ("    for (int ch = 0; ch < nch; ++ch) {", "    for (int ch = 0; ch < (PS_AGGW_PROBE == 1 ? 0 : nch); ++ch) {"),
    ]:
        assert old in tail, old
        tail = tail.replace(old, new, 1)
    return head + tail


def main():
    src = os.path.join(CSRC, "build", "aggw_probe.hip")
    with open(src, "w") as f:
        f.write(probe_source())
    objs = [o for o in glob.glob(os.path.join(CSRC, "build", "*.o")) if not o.endswith("aggw.o")
            and "aggw_p" not in o]
    for p in (1, 2):
        obj = os.path.join(CSRC, "build", f"aggw_p{p}.o")
        subprocess.check_call([HIPCC, "-std=c++17", "-O3", "--offload-arch=gfx950", "-fPIC", f"-DPS_AGGW_PROBE={p}",
                               "-I", CSRC, "-I", os.path.join(CSRC, "..", "..", "include"), "-c", src, "-o", obj])
        subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                               os.path.join(CSRC, "..", f"libpinsage_hip_p{p}.so"), *objs, obj, "-lpthread"])


if __name__ == "__main__":
    main()
