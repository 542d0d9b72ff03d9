# Round-6 half-frame hand-off A/B (ab/half1.so: -DXK_HALF lag 1, ab/half2.so: -DXK_HALF -DXK_LAG=2; cur = the
# shipped frame build): k_rdx parity tests of each variant, bench.py alternating (ms, sclk, checked legs against
# the fp64 oracle over every frame of the last step), then FETCH / WRITE per variant.
cd $GRAFT_REPO_ROOT
NOCOPY=1 TESTS="half1 half2" KEXPR="xcd and not deterministic" timeout -k 10 300 bash tools/gpu_r03_ab.sh "" 0 &&
AB="cur half1 half2" ROUNDS="1 2" timeout -k 10 700 bash tools/ab_bench.sh &&
timeout -k 10 300 bash tools/pmc_ab.sh "cur half1 half2"
