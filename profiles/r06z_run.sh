set -o pipefail
# BGP prefixes in the AllAreasRouteTable device tables: route table tests
D=gpurun_out/r06z; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_route_table.py > $D/gpu_tests.log 2>&1 || { tail -60 $D/gpu_tests.log; exit 3; }
tail -3 $D/gpu_tests.log
