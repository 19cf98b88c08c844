cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04l && mkdir -p $O
timeout -k 10 300 python tools/step_streams_bench.py --envs 262144 --splits 1,2,4,1 > $O/streams_262144.jsonl 2> $O/err1 || { echo failed; tail $O/err1; exit 1; }
cat $O/streams_262144.jsonl
timeout -k 10 300 python tools/step_streams_bench.py --envs 32768 --splits 1,2,4,1 > $O/streams_32768.jsonl 2> $O/err2 || { echo failed; tail $O/err2; exit 1; }
cat $O/streams_32768.jsonl
echo done
