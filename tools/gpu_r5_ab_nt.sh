set -u
cd "$GRAFT_REPO_ROOT"
bash tools/ab_libs.sh nt32 fp32 build/var_dwnt32.so build/var_mnt.so || exit $?
bash tools/ab_libs.sh mntbf bf16 build/var_mnt.so || exit $?
