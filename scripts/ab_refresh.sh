# Refresh ab_old/ (the B arm of scripts/ab_bench.sh) from the committed HEAD and build it.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$R/ab_old" && mkdir -p "$R/ab_old"
git -C "$R" archive HEAD | tar -x -C "$R/ab_old"
rm -rf "$R/ab_old/tests/golden" "$R/ab_old/profiles"
make -C "$R/ab_old/ducosy-gan_amd" -j8 >/dev/null
echo "ab_old = $(git -C "$R" rev-parse --short HEAD)"
