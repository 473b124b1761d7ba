#!/bin/bash
# round 3, GPU call 2: team tests (alignment), team-geometry x alignment decode-only A/B, encoder tile-partition A/B,
# and PMC traffic of the team kernel in both geometries.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -v -m gpu -k "team" --timeout 300 --timeout-method thread > $O/r03_tests_v2.log 2>&1
rc=$?
tail -5 $O/r03_tests_v2.log
[ $rc -le 1 ] || { echo "pytest rc=$rc: stopping"; exit $rc; }
for cfg in "0 0" "1 0" "1 1" "1 2" "0 2"; do
  set -- $cfg
  SKIP_GRAPH=1 TEAMS=8 LBIC_TEAM_XS=$1 LBIC_TEAM_ALIGN=$2 timeout -k 10 300 python -u tools/team_exp.py > $O/r03_teamexp_xs$1_al$2.log 2>&1 || exit 3
done
for swz in 0 2 1; do
  LBIC_ENC_SWZ=$swz timeout -k 10 300 python -u tools/enc_exp.py > $O/r03_encexp_swz$swz.log 2>&1 || exit 4
done
cd /tmp
for xs in 0 1; do
  rm -rf /tmp/tf$xs /tmp/th$xs
  TEAMS=8 SKIP_GRAPH=1 LBIC_TEAM_XS=$xs timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/tf$xs -o run -- python3 $R/tools/team_exp.py > $O/r03_team_pmc_fetch_xs$xs.log 2>&1 || exit 5
  TEAMS=8 SKIP_GRAPH=1 LBIC_TEAM_XS=$xs timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d /tmp/th$xs -o run -- python3 $R/tools/team_exp.py > $O/r03_team_pmc_hit_xs$xs.log 2>&1 || exit 6
  python3 $R/tools/pmc_summary.py $O/r03_team_pmc_xs$xs.json /tmp/tf$xs /tmp/th$xs > /dev/null || true
done
for swz in 0 2; do
  rm -rf /tmp/ef$swz
  LBIC_ENC_SWZ=$swz timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/ef$swz -o run -- python3 $R/tools/enc_exp.py > $O/r03_enc_pmc_fetch_swz$swz.log 2>&1 || exit 7
  python3 $R/tools/pmc_summary.py $O/r03_enc_pmc_swz$swz.json /tmp/ef$swz > /dev/null || true
done
cd $R
grep -h '"decoder"' $O/r03_teamexp_xs*_al*.log | cut -c1-200
cat $O/r03_encexp_swz*.log | cut -c1-300
echo done
