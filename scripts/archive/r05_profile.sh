#!/bin/bash
# Round-5 profile on one GPU box: the bench line + rocprof kernel trace + PMC passes of the stream
# workload (scripts/profile_round.sh), then the chain engine's own counters (scripts/engine_pmc.sh).
# Summaries: python scripts/summarize_profile.py <tag>; python scripts/summarize_engine_pmc.py <tag>_eng
cd $GRAFT_REPO_ROOT
TAG=${1:-r05prof}
bash scripts/profile_round.sh $TAG || exit $?
bash scripts/engine_pmc.sh ${TAG}_eng 6 || exit $?
echo done > gpurun_out/$TAG/ALL_DONE
