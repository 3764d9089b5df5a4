set -o pipefail
bash tools/g1.sh || exit 1
bash tools/g2.sh
