# Build the working tree as libcasr_hip_alt.so and HEAD as libcasr_hip.so (for ab_lib.sh)
set -e
cd "$(dirname "$0")/../.."
L=chinese-asr_amd/casr
python -c "import __graft_entry__ as g; g.build()" > /dev/null
cp $L/libcasr_hip.so /tmp/casr_alt.so
git stash -q
python -c "import __graft_entry__ as g; g.build()" > /dev/null || { git stash pop -q; exit 1; }
git stash pop -q
cp /tmp/casr_alt.so $L/libcasr_hip_alt.so
touch $L/libcasr_hip.so $L/libcasr_hip_alt.so
echo "base = HEAD, alt = working tree"
