# round 5: bench.py's live PMC traffic passes (N = 1, no extras)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5u; mkdir -p $O
( time timeout -k 10 400 python3 bench.py --no-extras > $O/bench.json 2> $O/bench.err ) 2> $O/time.txt || { tail -20 $O/bench.err; exit 1; }
cat $O/time.txt
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value']/1e9, d['roofline'])"
