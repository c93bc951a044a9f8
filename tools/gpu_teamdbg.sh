set -o pipefail
cd $GRAFT_REPO_ROOT
for v in "MANDO_TEAM=1" "MANDO_TEAM=2 MANDO_POA_DBG=8" "MANDO_TEAM=2" "MANDO_TEAM=8" "MANDO_TEAM=3"; do
  env $v timeout -k 10 200 python tools/team_dbg.py 3 2>&1 | grep -v "^\[" || exit 1
done
