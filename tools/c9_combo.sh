set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/c7_host.sh && bash tools/c8_rowfc.sh
