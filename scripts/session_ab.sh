#!/bin/bash
# Same-box A/B bench session: every line of $AB is "<name> <env assignments...> -- <bench.py args>",
# run in order (each its own `timeout`); JSON lines go to gpurun_out/bench_results.jsonl tagged
# with the name. Optional PROF="name ..." adds a rocprofv3 kernel-trace run of those entries.
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl" "$OUT/ab_results.jsonl"
while IFS= read -r line; do
  [ -z "$line" ] && continue
  name=${line%% *}; rest=${line#* }
  envs=${rest%%--*}; args=${rest#*--}
  step "ab_$name" 300 0 env $envs python bench.py $args
  grep -h '"metric"' "$OUT/ab_$name.log" | sed "s/^/{\"ab\": \"$name\", \"line\": /; s/\$/}/" >> "$OUT/ab_results.jsonl"
done <<< "$AB"
for name in $PROF; do
  line=$(grep "^$name " <<< "$AB"); rest=${line#* }; envs=${rest%%--*}; args=${rest#*--}
  cd /tmp && step "prof_$name" 300 0 env $envs rocprofv3 --kernel-trace --stats -d "$OUT/prof_$name" -o run \
    --output-format csv -- python3 "$ROOT/bench.py" $args --steps 5 --warmup 5; cd "$ROOT"
done
echo done
