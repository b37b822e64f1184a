LIBS="base nna" REPS=3 FINAL=base bash tools/gpurun_libab.sh || exit 1
for i in 1 2; do for q in 4 8; do
  RT_HW_QUEUES=$q timeout -k 10 120 python bench.py --no-cpu --steps 48 --emulate-ranks 8 > gpurun_out/hwq_$q$i.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('hwq', sys.argv[2], d['value'], d['ms_per_step'], d['config']['frames_in_flight'])" gpurun_out/hwq_$q$i.json $q
done; done
