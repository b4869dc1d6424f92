set -o pipefail
bash tools/ab_n_libs.sh nohalf1 "xsknf_amd/lib build/nohalf" 3 "1500 570 1024" || exit 1
