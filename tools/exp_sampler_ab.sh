# sampler A/B: the in-tree build against $PREV, interleaved (OUT file); also the scan's sampling
for r in 1 2; do
  for lib in base $PREV; do
    if [ "$lib" = base ]; then E=X=1; else E=ART_LIB=$lib; fi
    env $E timeout -k 10 200 python3 -u tools/exp_sampler_time.py 2>/dev/null | sed "s|^{|{\"lib\": \"$lib\", \"r\": $r, |" >> $OUT || exit 1
    env $E timeout -k 10 300 python3 -u tools/exp_scan_streams.py 1000000 8 32 16 2>/dev/null | tail -1 | sed "s|^{|{\"lib\": \"$lib\", \"r\": $r, \"scan\": 1, |" >> $OUT || exit 1
  done
done
