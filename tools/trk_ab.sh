set -e
for r in 1 2 3 4; do
  for v in ${VARIANTS:-trkbase trknf}; do
    YOUTH_ICP_LIB=tools/ab/$v/libyouth_icp.so timeout -k 10 120 python3 tools/stream_ab.py $v
  done
done
