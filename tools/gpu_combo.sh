# Development aid: run several A/B scripts in one box session (stops at the first failure).
set -o pipefail
cd $GRAFT_REPO_ROOT
for s in "$@"; do
  echo "=== $s"
  bash tools/$s || exit $?
done
