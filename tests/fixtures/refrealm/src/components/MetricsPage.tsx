import React, { useEffect, useState } from 'react';
import { SectionBox } from '@kinvolk/headlamp-plugin/lib/CommonComponents';
import { fetchGpuMetrics, formatWatts } from '../api/metrics';

// Fixture page: fetches in an effect, as the reference's Metrics page does.
export default function MetricsPage() {
  const [m, setM] = useState<any>(null);
  useEffect(() => {
    let cancelled = false;
    fetchGpuMetrics().then((r: any) => {
      if (!cancelled) setM(r);
    });
    return () => {
      cancelled = true;
    };
  }, []);
  return (
    <SectionBox title="Intel GPU — Metrics">
      {m ? <div>GPU Power Summary: {formatWatts(m.chips.length * 100)}</div> : <div>loading</div>}
    </SectionBox>
  );
}
