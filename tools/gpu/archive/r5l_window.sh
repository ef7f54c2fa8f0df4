# Sector-group gather window sweep (diagnostic): the multi-sector lower-PHY sweep at two UL/DL windows.
mkdir -p gpurun_out/r5n
for w in 100 300; do
  timeout -k 10 300 python -u tools/lower_phy_bench.py --sectors 2,4,6,8 --sweep-only gpu4,group0,group4,group13 \
    --window-us $w > gpurun_out/r5n/w$w.json 2> gpurun_out/r5n/w$w.log || exit 1
done
