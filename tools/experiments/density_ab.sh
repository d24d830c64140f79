for v in "QUEST_WAVE_CMIN=5 QUEST_WAVE_RELABEL=1" "QUEST_WAVE_CMIN=5 QUEST_WAVE_RELABEL=0" "QUEST_WAVE_CMIN=6 QUEST_WAVE_RELABEL=0" "QUEST_WAVE_CMIN=6 QUEST_WAVE_RELABEL=1" "QUEST_WAVE_CMIN=4 QUEST_WAVE_RELABEL=1"; do
  echo "$v $(env $v timeout -k 10 200 python tools/bench_suite.py --only density17 2>&1 | grep '^density17')"
done
