python bench.py --no-cpu --no-configs --steps 30 | python3 -c "import json,sys; d=json.load(sys.stdin); print('%.4f' % d['ms_per_step'], ['%.4f' % x for x in d['roofline']['pass_ms']])"
