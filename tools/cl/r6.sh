# Round 6 GPU calls, one case per gpurun call: bash tools/cl/r6.sh <case>
# (every step is tools/gpu.sh; results under gpurun_out/r6/<case>/, copied to profiles/r6/)
set -o pipefail
G="bash tools/gpu.sh"
C=r6/$1
# configs[3]'s 8 bands at the round-5 last build's measured cut (profiles/r5/bands/last_build_recut.jsonl)
B5='[[0, 572], [572, 750], [750, 895], [895, 1059], [1059, 1281], [1281, 1534], [1534, 1778], [1778, 2160]]'
case "$1" in
first)  # the round's first build: suite, smoke, headline + C1 ReSTIR lines, shipped-library profile, bands
    $G suite $C && $G smoke $C &&
    $G bench $C reuse && $G bench $C restir --workload restir --no-configs3 &&
    $G profile $C/prof_reuse && $G bands $C bands_r5cut --world 8 --bands "$B5" ;;
*)
    echo "unknown case $1"; exit 2 ;;
esac
