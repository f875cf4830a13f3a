cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for p in 0 0 1 1; do
  DOCQA_GROUP_PERSIST=$p timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_rag_pipelined.py -k gpu 2>&1 | tail -2 | head -1 | sed "s/^/[persist=$p] /"
done
