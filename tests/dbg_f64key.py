# temporary GPU debug helper (not a test)
import sys, numpy as np
sys.path.insert(0,'.'); sys.path.insert(0,'query-engines_amd')
from kquery import native as N
from kquery.columnar import DeviceColumn, Context
from kquery.aggregate import HashAggregateState
ctx=Context.get(0)
k=np.array([0.0,-0.0,1.5,-0.0,np.nan,-0.0])
st=HashAggregateState(ctx,[N.TYPE_FLOAT64],[(N.AGG_COUNT_STAR,N.TYPE_INT64)],16)
st.update([DeviceColumn.from_numpy(N.TYPE_FLOAT64,k,ctx=ctx)],[None])
print('groups',st.num_groups())
kk,aa=st.finalize()
print(kk[0].to_pylist(), aa[0].to_pylist(), kk[0].valid_mask())
